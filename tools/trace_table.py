#!/usr/bin/env python3
"""Per-kernel table of a rocprofv3 --kernel-trace directory: calls, mean duration, and the launch
geometry (grid, workgroup, LDS, VGPRs), heaviest first.

usage: python tools/trace_table.py TRACE_DIR [N]
"""
import collections
import csv
import glob
import sys


def main():
    f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    rows = list(csv.DictReader(open(f)))
    agg = collections.defaultdict(list)
    for r in rows:
        k = r["Kernel_Name"].split("(")[0][:80]
        key = (k, r.get("Grid_Size_X", r.get("Grid_Size")), r.get("Workgroup_Size_X", r.get("Workgroup_Size")),
               r.get("LDS_Block_Size"), r.get("VGPR_Count"))
        agg[key].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    print("calls  mean_us  total_us  kernel / grid / wg / lds / vgpr")
    for k, v in sorted(agg.items(), key=lambda x: -sum(x[1]))[:n]:
        print(f"{len(v):5d} {sum(v) / len(v) / 1000:8.1f} {sum(v) / 1000:9.1f}  {k}")


if __name__ == "__main__":
    main()
