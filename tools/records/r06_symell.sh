#!/bin/bash
# symbolic MODE 4 over B in CSR form building B's ELL image (no k_build_ell launch first): stored /
# spgemm / spec / tiny / graph / magnus tests, headline + chain A/B against SLAT_NO_SYM_ELL, headline trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r06symell}; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests/test_stored_mode_gpu.py tests/test_spgemm_gpu.py tests/test_f64_any_order_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -v "^  File\|^    " $OUT/pytest.log | tail -30; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 400 python3 tools/ab.py --reps 2 --chain --sat64 tree knobs:SLAT_NO_SYM_ELL=1 > $OUT/ab.txt 2>&1 || { tail $OUT/ab.txt; exit 1; }
tail -3 $OUT/ab.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/ht -o head --output-format csv -- python3 tools/prof_head.py > $OUT/ht.log 2>&1 || { tail $OUT/ht.log; exit 1; }
grep headline $OUT/ht.log
python3 tools/trace_table.py $OUT/ht 5
python3 tools/trace_gaps.py $OUT/ht 9
