#!/bin/bash
# lane path: 64 vs 32 rows per block (k11 / k11r32); fold-order fat walk with / without the next
# groups' loads in flight (k11 / nopf); the parity tests of both first
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r04ab8}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_spgemm_gpu.py tests/test_fat_rows_gpu.py tests/test_f64_any_order_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -n 2 $OUT/pytest.log
SLAT_LIB_PATH=$GRAFT_REPO_ROOT/tools/var/libslat_k11r32.so timeout -k 10 300 python -u -m pytest tests/test_spgemm_gpu.py -k lane -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_r32.log 2>&1 || { tail -40 $OUT/pytest_r32.log; exit 1; }
tail -n 1 $OUT/pytest_r32.log
timeout -k 10 400 python tools/ab.py --reps 3 --steps 200 --chain k11 k11r32 > $OUT/ab.txt 2>&1 || { tail -30 $OUT/ab.txt; exit 1; }
grep -A3 summary $OUT/ab.txt | cut -c1-400
timeout -k 10 900 python tools/ab_heavy.py --reps 2 --big --legs c5ord,c5big_ord nopf k11 > $OUT/heavy.txt 2>&1 || { tail -30 $OUT/heavy.txt; exit 1; }
tail -n 3 $OUT/heavy.txt | cut -c1-900
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 tools/ab.py --child --steps 40 --chain > $OUT/child.json 2> $OUT/child.err || { tail -20 $OUT/child.err; exit 1; }
python3 tools/trace_table.py $OUT/trace 12 > $OUT/trace_table.txt && cat $OUT/trace_table.txt
