#!/bin/bash
# lane kernel: structural count before the look-back, zero sums compacted by the host (k14) vs k13;
# phases of the new build; parity first
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r04ab10}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_spgemm_gpu.py tests/test_tiny_gpu.py tests/test_graph_gpu.py tests/test_coo_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -n 2 $OUT/pytest.log
timeout -k 10 400 python tools/ab.py --reps 3 --steps 200 --chain k13 k14 > $OUT/ab.txt 2>&1 || { tail -30 $OUT/ab.txt; exit 1; }
grep -A3 summary $OUT/ab.txt | cut -c1-300
SLAT_LIB_PATH=$GRAFT_REPO_ROOT/tools/var/libslat_ph.so timeout -k 10 120 python tools/phases_chain.py 3 > $OUT/phases.txt 2>&1 || { tail -20 $OUT/phases.txt; exit 1; }
head -6 $OUT/phases.txt
