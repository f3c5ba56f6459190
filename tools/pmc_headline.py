#!/usr/bin/env python3
"""profiles/rNN_pmc_torus30_a7.json from one tools/prof_pmc.sh run (FETCH_SIZE pass, WRITE_SIZE pass):
per kernel of the headline step the bytes of its LAST dispatch (a timed bench step), FETCH_SIZE x 1024
x 2 (gfx950 half-count correction, MI355X_MICROARCH.md HBM section), WRITE_SIZE x 1024. bench.py reads
the newest such file for roofline.traffic.

usage: pmc_headline.py PROF_DIR ROUND_TAG > profiles/<tag>_pmc_torus30_a7.json"""
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import load, short  # noqa: E402


def main():
    d, tag = sys.argv[1], sys.argv[2]
    last = load(glob.glob(os.path.join(d, "pmc*", "**", "*counter_collection.csv"), recursive=True))
    per = {}
    for k, c in last.items():
        if "slat" not in k:
            continue
        r = {"read_bytes_corrected": c.get("FETCH_SIZE", 0.0) * 1024 * 2, "write_bytes": c.get("WRITE_SIZE", 0.0) * 1024,
             "dur_ns": c.get("_dur_ns")}
        r["bytes"] = r["read_bytes_corrected"] + r["write_bytes"]
        per[short(k)] = r
    num = [k for k in per if "k_numeric<" in k]
    sym = [k for k in per if "k_symbolic<" in k]
    out = {"workload": "torus30_a7", "round": tag,
           "kernel": num[0] if num else None,
           "numeric_bytes_per_launch": int(per[num[0]]["bytes"]) if num else None,
           "read_bytes_corrected": int(per[num[0]]["read_bytes_corrected"]) if num else None,
           "write_bytes": int(per[num[0]]["write_bytes"]) if num else None,
           "symbolic_bytes_per_launch": int(per[sym[0]]["bytes"]) if sym else None,
           "pipeline_bytes_per_step": int(sum(v["bytes"] for v in per.values())),
           "per_kernel": per,
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes (tools/prof_pmc.sh) of "
                     "bench.py --no-c4 --steps 3 --warmup 1; last dispatch per kernel; FETCH_SIZE x1024 x2 (gfx950), "
                     "WRITE_SIZE x1024",
           "source_run": d}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
