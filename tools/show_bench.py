import json, sys
d = json.load(open(sys.argv[2]))
print(sys.argv[1], d["value"], d["roofline"]["kernel_ms"], "ablated_ms=%s" % d["config"].get("ablated_ms"))
