#!/usr/bin/env python3
"""Summarise a bench.py rocprofv3 run for profiles/.

usage: prof_summary.py TRACE_DIR STEPS [PMC_SUMMARY_JSON] > profiles/rNN_<workload>.md

Per-kernel duration statistics over the last STEPS timed steps only (a step starts at a
k_build_ell or k_symbolic dispatch), so the averages are comparable with bench.py's HIP-event
kernel_ms; the whole-run rocprofv3 --stats table (which also holds the A^2..A^6 input-building
calls) is appended verbatim, and the PMC HBM bytes per launch when a pmc summary is given.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(k):
    k = k.replace("void ", "")
    if "rocprim" in k:
        return "rocprim::" + ("init_lookback_scan_state" if "init_lookback" in k else "scan (hipcub InclusiveSum)")
    return k.split("(")[0]


def main():
    tdir, steps = sys.argv[1], int(sys.argv[2])
    pmc = json.load(open(sys.argv[3])) if len(sys.argv) > 3 else None
    trace = glob.glob(os.path.join(tdir, "**", "*kernel_trace.csv"), recursive=True)[0]
    stats = glob.glob(os.path.join(tdir, "**", "*kernel_stats.csv"), recursive=True)[0]
    rows = list(csv.DictReader(open(trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows)
              if "k_build_ell" in r["Kernel_Name"] or
              ("k_symbolic" in r["Kernel_Name"] and (i == 0 or "k_build_ell" not in rows[i - 1]["Kernel_Name"]))]
    first = starts[-steps]
    timed = rows[first:]
    dur = defaultdict(list)
    for r in timed:
        dur[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    span = (int(timed[-1]["End_Timestamp"]) - int(timed[0]["Start_Timestamp"])) / 1e3
    print(f"# rocprofv3 kernel trace, last {steps} timed steps\n")
    print(f"trace: `{os.path.relpath(trace)}`; wall span of the timed dispatches {span:.1f} us "
          f"({span / steps:.1f} us/step incl. host gaps)\n")
    print("| kernel | calls | avg us | min us | max us | us/step |")
    print("|---|---|---|---|---|---|")
    for k, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        print(f"| `{k}` | {len(v)} | {sum(v) / len(v):.2f} | {min(v):.2f} | {max(v):.2f} | {sum(v) / steps:.2f} |")
    if pmc:
        print("\n## PMC (separate --pmc passes, last dispatch of each kernel)\n")
        print("| kernel | FETCH_SIZE KiB | HBM read B (x2 gfx950 correction) | WRITE_SIZE B | total B |")
        print("|---|---|---|---|---|")
        for k, c in sorted(pmc.items()):
            rd, wr = c.get("hbm_read_bytes_corrected"), c.get("hbm_write_bytes")
            tot = (rd or 0) + (wr or 0)
            print(f"| `{k}` | {c.get('FETCH_SIZE', '')} | {rd:.0f} | {wr:.0f} | {tot:.0f} |")
    print("\n## rocprofv3 --kernel-trace --stats (whole run, includes input-building calls)\n")
    print("```")
    print(open(stats).read().rstrip())
    print("```")


if __name__ == "__main__":
    main()
