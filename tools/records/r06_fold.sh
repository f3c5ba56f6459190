#!/bin/bash
# folded row offsets v2 (atomic first/second-level words, no k_scan_rows): fold / stored / spgemm /
# spec / wide / prepared / dist / tiny tests, the headline + chain A/B against the knobs build with
# SLAT_NO_FOLD, then C4 whole against one eighth (tree, and SLAT_NO_FOLD)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r06fold}; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests/test_fold_gpu.py tests/test_stored_mode_gpu.py tests/test_spgemm_gpu.py tests/test_spec_wide_gpu.py tests/test_wide_hash_gpu.py tests/test_prepared_gpu.py tests/test_dist_hip_gpu.py tests/test_tiny_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -v "^  File\|^    " $OUT/pytest.log | tail -30; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 400 python3 tools/ab.py --reps 2 --chain --sat64 tree knobs:SLAT_NO_FOLD=1 > $OUT/ab.txt 2>&1 || { tail $OUT/ab.txt; exit 1; }
tail -3 $OUT/ab.txt
for v in tree nofold tree nofold; do
  if [ $v = tree ]; then timeout -k 10 120 python3 tools/c4_eighth.py; else SLAT_LIB_PATH=tools/var/libslat_knobs.so SLAT_NO_FOLD=1 timeout -k 10 120 python3 tools/c4_eighth.py; fi > $OUT/c4_$v.txt 2>&1 || { tail $OUT/c4_$v.txt; exit 1; }
  echo "$v $(cat $OUT/c4_$v.txt)"
done
