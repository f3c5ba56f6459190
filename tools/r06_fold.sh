#!/bin/bash
# folded row offsets (MODE 4 without k_scan_rows): fold / stored / spgemm / spec / wide tests, then the
# headline + chain A/B: tree, the knobs build with SLAT_NO_FOLD, and the previous build (spec1)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r06fold}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_fold_gpu.py tests/test_stored_mode_gpu.py tests/test_spgemm_gpu.py tests/test_spec_wide_gpu.py tests/test_tiny_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -v "^  File\|^    " $OUT/pytest.log | tail -30; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 400 python3 tools/ab.py --reps 2 --chain --sat64 tree knobs:SLAT_NO_FOLD=1 spec1 > $OUT/ab.txt 2>&1 || { tail $OUT/ab.txt; exit 1; }
tail -4 $OUT/ab.txt
