#!/bin/bash
# C5 2^18 (any order, then fold order): kernel traces
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r05c5}; mkdir -p $OUT
for leg in c5big_any c5big_ord; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$leg -o $leg --output-format csv -- python3 tools/ab_heavy.py --child --big --legs $leg > $OUT/$leg.log 2>&1 || { tail $OUT/$leg.log; exit 1; }
tail -1 $OUT/$leg.log | cut -c1-300
python3 tools/trace_table.py $OUT/$leg 12
done
