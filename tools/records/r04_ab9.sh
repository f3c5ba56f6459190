#!/bin/bash
# lane path: payload-free key sort (k12) and the wave look-back (k13) against each other; the small
# cells (tiny kernel with the wave look-back); parity first
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r04ab9}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_spgemm_gpu.py tests/test_tiny_gpu.py tests/test_graph_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -n 2 $OUT/pytest.log
timeout -k 10 400 python tools/ab.py --reps 3 --steps 200 --chain k12 k13 r3 > $OUT/ab.txt 2>&1 || { tail -30 $OUT/ab.txt; exit 1; }
grep -A4 summary $OUT/ab.txt | cut -c1-300
timeout -k 10 300 python tools/small_cells.py > $OUT/small_cells.txt 2>&1 || { tail -30 $OUT/small_cells.txt; exit 1; }
tail -25 $OUT/small_cells.txt
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 tools/ab.py --child --steps 40 --chain > $OUT/child.json 2> $OUT/child.err || { tail -20 $OUT/child.err; exit 1; }
python3 tools/trace_table.py $OUT/trace 8 > $OUT/trace_table.txt && cat $OUT/trace_table.txt
