#!/bin/bash
# the GPU suite on the tree, C4 whole vs eighths, the heavy legs against round 4's library
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r05c3}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 120 python3 tools/c4_eighth.py > $OUT/c4_eighth.json 2>&1 || { tail $OUT/c4_eighth.json; exit 1; }
cat $OUT/c4_eighth.json
timeout -k 10 400 python3 tools/ab_heavy.py --reps 2 --legs rg,c5any,c5ord,chain tree base4 > $OUT/heavy.txt 2>&1 || { tail $OUT/heavy.txt; exit 1; }
tail -3 $OUT/heavy.txt
timeout -k 10 200 python3 bench.py --no-cpu --e2e-steps 0 --no-c4 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
cut -c1-400 $OUT/bench.json
