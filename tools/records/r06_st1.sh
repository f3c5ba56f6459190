#!/bin/bash
# MODE 4 (stored-bitmap numeric) first check: its tests + the spgemm suite, then A/B against MODE 0
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r06st1}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_stored_mode_gpu.py tests/test_spgemm_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 400 python3 tools/ab.py --reps 2 --sat64 --chain knobs knobs:SLAT_NO_STORED_MODE=1 > $OUT/ab.txt 2>&1 || { tail $OUT/ab.txt; exit 1; }
cat $OUT/ab.txt
