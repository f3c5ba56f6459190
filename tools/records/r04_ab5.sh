#!/bin/bash
# short rows of wide CSR-B launches batched (k7) against one row per table (SLAT_NO_CSR_BATCH=1), the
# fat threshold by B form, the single-window short rows off again: GPU suite parts, chain, heavy
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r04ab5}; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest ${TESTS:-tests/test_spgemm_gpu.py tests/test_fat_rows_gpu.py tests/test_f64_any_order_gpu.py tests/test_real_graph_gpu.py tests/test_short_sort_gpu.py tests/test_graph_gpu.py tests/test_tiny_gpu.py} -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -n 2 $OUT/pytest.log
timeout -k 10 500 python tools/ab.py --reps 2 --steps 100 --chain --c4 r3 k7 > $OUT/ab.txt 2>&1 || { tail -30 $OUT/ab.txt; exit 1; }
grep -A3 summary $OUT/ab.txt | cut -c1-800
timeout -k 10 900 python tools/ab_heavy.py --reps 1 --big r3 k7 k7:SLAT_NO_CSR_BATCH=1 > $OUT/heavy.txt 2>&1 || { tail -30 $OUT/heavy.txt; exit 1; }
tail -n 4 $OUT/heavy.txt | cut -c1-900
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/htrace -o run --output-format csv -- python3 tools/ab_heavy.py --child --legs rg,c5any > $OUT/hchild.json 2> $OUT/hchild.err || { tail -20 $OUT/hchild.err; exit 1; }
cat $OUT/hchild.json
python3 tools/trace_table.py $OUT/htrace > $OUT/htrace_table.txt && head -25 $OUT/htrace_table.txt
