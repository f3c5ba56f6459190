#!/bin/bash
# SQ instruction-mix counters of the C4 kernels (one --pmc pass, kernel trace only)
set -o pipefail
OUT=gpurun_out/r02_pmc_c4
mkdir -p $OUT
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS -d $OUT/p1 -o c4 --output-format csv -- python3 tools/prof_c4.py > $OUT/p1.log 2>&1 || { tail $OUT/p1.log; exit 1; }
f=$(find $OUT/p1 -name "*counter_collection.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"][:60]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    n[(k, r["Counter_Name"])] += 1
for k, d in acc.items():
    if "short" in k or "k_numeric" in k or "symbolic" in k:
        print(k, {c: f"{v:.3g}" for c, v in d.items()})
PY
