#!/bin/bash
# SQ stall / instruction-mix / LDS counters of the bench's kernels (30^3 A^6*A): two --pmc passes,
# each its own run (kernel trace only), summarised per kernel over the timed steps' dispatches
set -o pipefail
OUT=gpurun_out/r02_pmc_bench
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
i=0
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C -d $OUT/p$i -o run --output-format csv -- python3 bench.py --no-cpu --steps 3 --warmup 1 > $OUT/p$i.log 2>&1 || { tail $OUT/p$i.log; exit 1; }
done
python3 - $OUT <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
last = collections.defaultdict(dict)
for f in glob.glob(f"{out}/p*/**/*counter_collection.csv", recursive=True):
    disp = collections.defaultdict(dict)
    for r in csv.DictReader(open(f)):
        disp[(r["Kernel_Name"], int(r["Dispatch_Id"]))][r["Counter_Name"]] = float(r["Counter_Value"])
    for (k, d), c in sorted(disp.items(), key=lambda x: x[0][1]):
        last[k].update(c)  # the last dispatch of each kernel: a timed step
for k, c in last.items():
    if any(s in k for s in ("k_numeric", "k_symbolic", "k_build_ell", "k_scan")):
        print(k.split("(")[0][:70])
        for n in sorted(c):
            print(f"   {n:24s} {c[n]:.4g}")
PY
