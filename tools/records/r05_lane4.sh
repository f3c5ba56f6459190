#!/bin/bash
# the lane kernel's quad-parallel count and combine: its tests, C1 per call, the phase split
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r05lane4}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_spgemm_gpu.py tests/test_tiny_gpu.py -x -q --timeout 120 --timeout-method thread -k "lane or tiny or torus30 or sweep or zero or satur or pattern" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for i in 1 2 3; do timeout -k 10 120 python3 tools/prof_c1.py >> $OUT/c1.out 2>&1 || { tail $OUT/c1.out; exit 1; }; done
cat $OUT/c1.out
SLAT_LIB_PATH=tools/var/libslat_phases.so timeout -k 10 120 python3 tools/prof_c1.py > $OUT/phases.out 2> $OUT/phases.log || { tail $OUT/phases.log; exit 1; }
tail -1 $OUT/phases.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/trace -o c1 --output-format csv -- python3 tools/prof_c1.py > $OUT/prof.log 2>&1 || { tail $OUT/prof.log; exit 1; }
find $OUT/trace -name "*kernel_stats.csv" -exec head -3 {} \;
