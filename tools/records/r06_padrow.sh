#!/bin/bash
# ELL padding row; MODE 4 symbolic group loads without a branch per entry (numeric keeps its branches): stored / spgemm / f64-any /
# magnus tests, then the headline + chain + Sat64 A/B against the committed build (knobs, no env)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r06padrow2}; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests/test_stored_mode_gpu.py tests/test_spec_wide_gpu.py tests/test_spgemm_gpu.py tests/test_f64_any_order_gpu.py tests/test_magnus_usize_gpu.py tests/test_fat_rows_gpu.py tests/test_prepared_gpu.py tests/test_wide_hash_gpu.py tests/test_short_sort_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -v "^  File\|^    " $OUT/pytest.log | tail -30; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 500 python3 tools/ab.py --reps 3 --chain --sat64 tree base > $OUT/ab.txt 2>&1 || { tail $OUT/ab.txt; exit 1; }
tail -3 $OUT/ab.txt
