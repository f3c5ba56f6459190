#!/bin/bash
# Round-3 call ai: the GPU suite on the final tree; where a small call's ~22 us goes: the host split (SLAT_HOST_CLOCK=1) of the 4^3
# torus A*A (one kernel) and a kernel trace of the small cells
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03ai; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -n 1 $OUT/pytest.log
SLAT_HOST_CLOCK=1 timeout -k 10 300 python tools/host_overhead.py > $OUT/host.txt 2>&1 || { tail -30 $OUT/host.txt; exit 1; }
grep -E "host us|tiny|step" $OUT/host.txt | tail -6
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/sc -o sc --output-format csv -- python3 tools/small_cells.py > $OUT/sc.log 2>&1 || { tail -20 $OUT/sc.log; exit 1; }
echo done
