#!/bin/bash
# the one-kernel lane path for short-row products: its parity tests first (one process), then the
# 30^3 chain against round 3's library
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r04lane1}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_spgemm_gpu.py -k "lane" -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_lane.log 2>&1 || { tail -40 $OUT/pytest_lane.log; exit 1; }
tail -n 2 $OUT/pytest_lane.log
timeout -k 10 600 python -u -m pytest tests/test_spgemm_gpu.py tests/test_tiny_gpu.py tests/test_graph_gpu.py tests/test_dropin_cpp_gpu.py tests/test_magnus_usize_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -n 2 $OUT/pytest.log
timeout -k 10 500 python tools/ab.py --reps 2 --steps 100 --chain r3 k10 k10:SLAT_NO_LANE=1 > $OUT/ab.txt 2>&1 || { tail -30 $OUT/ab.txt; exit 1; }
grep -A4 summary $OUT/ab.txt | cut -c1-800
