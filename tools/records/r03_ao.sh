#!/bin/bash
# Round-3 closing call: smoke, the default bench line and the multi-rank rehearsal on one GPU
# (dist tests, RCCL at world size 1 with the C4 leg's parity, 2 gloo ranks) on the final tree
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03ao; mkdir -p $OUT
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 240 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
bash tools/r02_dist.sh r03ao/dist || exit 1
echo done
