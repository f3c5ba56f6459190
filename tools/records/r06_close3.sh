#!/bin/bash
# round-6 closing check of the committed tree (last session): the GPU suite, smoke(), the driver's bench
# command, and a kernel trace with stats of that command, each step under its own time limit
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r06close3; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -v "^  File\|^    " $OUT/pytest.log | tail -40; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
tail -c 600 $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/tr -o drv --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --e2e-steps 0 > $OUT/tr.log 2>&1 || { tail $OUT/tr.log; exit 1; }
find $OUT/tr -name "*kernel_stats.csv" | head -3
