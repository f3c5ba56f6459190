#!/bin/bash
# the headline step: k_numeric's phase split (variant build) and a kernel trace of a short bench run
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r05head}; mkdir -p $OUT
SLAT_LIB_PATH=tools/var/libslat_phases.so timeout -k 10 120 python3 tools/phases_a7.py 6 > $OUT/phases.log 2>&1 || { tail $OUT/phases.log; exit 1; }
tail -4 $OUT/phases.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/trace -o a7 --output-format csv -- python3 bench.py --steps 40 --warmup 20 --no-cpu --no-c4 --e2e-steps 0 > $OUT/bench.log 2>&1 || { tail $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-300
