#!/bin/bash
# calls returning after their scan (zero-free operands): the early-return tests and the suites that run
# chains and row blocks, then the headline + chain A/B against SLAT_NO_EARLY, C4 whole / eighth, and
# the headline trace with its per-dispatch gaps
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r06early}; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests/test_early_return_gpu.py tests/test_spgemm_gpu.py tests/test_spec_wide_gpu.py tests/test_prepared_gpu.py tests/test_dist_hip_gpu.py tests/test_graph_gpu.py tests/test_coo_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -v "^  File\|^    " $OUT/pytest.log | tail -30; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 400 python3 tools/ab.py --reps 2 --chain --sat64 tree knobs:SLAT_NO_EARLY=1 > $OUT/ab.txt 2>&1 || { tail $OUT/ab.txt; exit 1; }
tail -3 $OUT/ab.txt
for v in tree noearly; do
  if [ $v = tree ]; then timeout -k 10 120 python3 tools/c4_eighth.py; else SLAT_LIB_PATH=tools/var/libslat_knobs.so SLAT_NO_EARLY=1 timeout -k 10 120 python3 tools/c4_eighth.py; fi > $OUT/c4_$v.txt 2>&1 || { tail $OUT/c4_$v.txt; exit 1; }
  echo "$v $(cat $OUT/c4_$v.txt)"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/ht -o head --output-format csv -- python3 tools/prof_head.py > $OUT/ht.log 2>&1 || { tail $OUT/ht.log; exit 1; }
grep headline $OUT/ht.log
python3 tools/trace_gaps.py $OUT/ht 8
