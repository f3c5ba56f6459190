#!/usr/bin/env python3
"""Print the last N kernel dispatches of a rocprofv3 kernel-trace CSV with durations."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 12
last = rows[-n:]
t0 = int(last[0]["Start_Timestamp"])
for r in last:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print(f"{s/1000:9.2f} {(e-s)/1000:8.2f}us  {r['Kernel_Name'][:70]}")
