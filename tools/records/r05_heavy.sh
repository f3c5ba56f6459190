#!/bin/bash
# the heavy legs (power-law inputs) against round 4's library, then the parity suites that cover them
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r05hv}; mkdir -p $OUT
timeout -k 10 400 python3 tools/ab_heavy.py --reps 2 --legs rg,c5any,c5ord,chain tree base4 > $OUT/heavy.txt 2>&1 || { tail $OUT/heavy.txt; exit 1; }
tail -3 $OUT/heavy.txt
timeout -k 10 300 python -u -m pytest tests/test_fat_rows_gpu.py tests/test_wide_hash_gpu.py tests/test_short_sort_gpu.py tests/test_real_graph_gpu.py tests/test_prepared_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 120 python3 tools/c4_eighth.py > $OUT/c4_eighth.json 2>&1 || { tail $OUT/c4_eighth.json; exit 1; }
cat $OUT/c4_eighth.json
