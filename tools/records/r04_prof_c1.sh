#!/bin/bash
# C1 (the lane kernel): kernel trace, then FETCH / WRITE and SQ counter passes, each its own run
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r04c1}; mkdir -p $OUT
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/trace -o c1 --output-format csv -- python3 tools/prof_c1.py > $OUT/trace.log 2>&1 || { tail $OUT/trace.log; exit 1; }
grep "C1:" $OUT/trace.log
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc1 -o c1 --output-format csv -- python3 tools/prof_c1.py > $OUT/pmc1.log 2>&1 || { tail $OUT/pmc1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc2 -o c1 --output-format csv -- python3 tools/prof_c1.py > $OUT/pmc2.log 2>&1 || { tail $OUT/pmc2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS -d $OUT/pmc3 -o c1 --output-format csv -- python3 tools/prof_c1.py > $OUT/pmc3.log 2>&1 || { tail $OUT/pmc3.log; exit 1; }
python3 tools/pmc_summary.py "$OUT/pmc*/**/*counter_collection.csv" > $OUT/c1_pmc.json && head -c 1200 $OUT/c1_pmc.json
