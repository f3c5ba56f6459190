#!/bin/bash
# the GPU suite, then C1 (the lane kernel) traced and timed, and C4 whole vs eighths
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r05lane}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/c1trace -o c1 --output-format csv -- python3 tools/prof_c1.py > $OUT/c1trace.log 2>&1 || { tail $OUT/c1trace.log; exit 1; }
grep "C1" $OUT/c1trace.log | tail -1
grep k_lane $OUT/c1trace/*kernel_stats.csv | cut -c1-200
timeout -k 10 120 python3 tools/prof_c1.py 2>&1 | tail -1
timeout -k 10 120 python3 tools/c4_eighth.py > $OUT/c4_eighth.json 2>&1 || { tail $OUT/c4_eighth.json; exit 1; }
cat $OUT/c4_eighth.json
