#!/bin/bash
# usage: tools/prof_pmc.sh OUTDIR "bench args" "COUNTERS_1" ["COUNTERS_2" ...]
# One rocprofv3 --kernel-trace --stats pass, then one --pmc pass per counter group.
set -e
OUT=$1; shift
ARGS=$1; shift
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --no-cpu $ARGS > $OUT/bench.json 2> $OUT/bench.err
i=0
for C in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $C -d $OUT/pmc$i -o run --output-format csv -- python3 bench.py --no-cpu --steps 3 --warmup 1 $ARGS > /dev/null 2>> $OUT/pmc.err
done
echo done
