#!/bin/bash
# FETCH_SIZE / WRITE_SIZE and the SQ wave counters of the heavy products' kernels (RG R-MAT 2^16 A^2
# u32, C5 R-MAT 2^16 f64 any order), one --pmc pass per (leg, counter group), each its own run
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r04hp}; mkdir -p $OUT
for LEG in ${LEGS:-rg c5any}; do
  i=0
  for C in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU"; do
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --pmc $C -d $OUT/$LEG/pmc$i -o run --output-format csv -- python3 tools/ab_heavy.py --child --legs $LEG > $OUT/$LEG.pmc$i.json 2>> $OUT/pmc.err || { tail -20 $OUT/pmc.err; exit 1; }
  done
  python3 tools/pmc_summary.py "$OUT/$LEG/pmc*/**/*counter_collection.csv" > $OUT/pmc_$LEG.json && head -c 2500 $OUT/pmc_$LEG.json
done
