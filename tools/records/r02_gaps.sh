#!/bin/bash
# kernel trace of the headline bench: per-kernel times and the gaps between consecutive dispatches
set -o pipefail
OUT=gpurun_out/r02_gaps
mkdir -p $OUT
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/t -o run -- python3 bench.py --no-cpu --steps 200 --warmup 50 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
f=$(find $OUT/t -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))[-500:]
gaps, durs, prev = collections.defaultdict(list), collections.defaultdict(list), None
for r in rows:
    n = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "").replace("slat::", "")
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    durs[n].append((e - s) / 1e3)
    if prev: gaps[(prev[0], n)].append((s - prev[1]) / 1e3)
    prev = (n, e)
for k, v in durs.items(): print("dur", k, len(v), "median %.2f us" % sorted(v)[len(v) // 2])
for k, v in gaps.items(): print("gap", k, len(v), "median %.2f us" % sorted(v)[len(v) // 2])
PY
