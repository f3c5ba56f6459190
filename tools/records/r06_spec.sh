#!/bin/bash
# speculative wide launches + the MODE 4 numeric with the next row's loads ahead: their tests and the
# wide / prepared / dist / stored / spgemm suites, the headline A/B against the previous build, C4
# whole against one eighth (tree, and the knobs build with SLAT_NO_SPEC)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r06spec}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_spec_wide_gpu.py tests/test_wide_hash_gpu.py tests/test_prepared_gpu.py tests/test_dist_hip_gpu.py tests/test_stored_mode_gpu.py tests/test_spgemm_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -v "^  File\|^    " $OUT/pytest.log | tail -30; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 300 python3 tools/ab.py --reps 2 --chain tree spec1 > $OUT/ab.txt 2>&1 || { tail $OUT/ab.txt; exit 1; }
tail -3 $OUT/ab.txt
for v in tree nospec tree nospec; do
  if [ $v = tree ]; then timeout -k 10 120 python3 tools/c4_eighth.py; else SLAT_LIB_PATH=tools/var/libslat_knobs.so SLAT_NO_SPEC=1 timeout -k 10 120 python3 tools/c4_eighth.py; fi > $OUT/c4_$v.txt 2>&1 || { tail $OUT/c4_$v.txt; exit 1; }
  echo "$v $(cat $OUT/c4_$v.txt)"
done
