#!/usr/bin/env python3
"""Timeline of the last N dispatches of a rocprofv3 --kernel-trace directory: kernel, duration, and
the gap since the previous dispatch ended (where a call's fixed costs hide between its launches).

usage: python tools/trace_gaps.py TRACE_DIR [N]
"""
import csv
import glob
import sys


def main():
    f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    prev = None
    print("   start_us   dur_us   gap_us  grid  kernel")
    t0 = int(rows[-n]["Start_Timestamp"]) if len(rows) >= n else int(rows[0]["Start_Timestamp"])
    for r in rows[-n:]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev) / 1000 if prev is not None else 0.0
        prev = e
        k = r["Kernel_Name"].split("(")[0][-60:]
        g = r.get("Grid_Size_X", r.get("Grid_Size"))
        print(f"{(s - t0) / 1000:11.1f} {(e - s) / 1000:8.1f} {gap:8.1f} {g:>6}  {k}")


if __name__ == "__main__":
    main()
