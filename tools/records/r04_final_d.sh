#!/bin/bash
# Round-4 final tree (second record): tools/r04_check.sh, one rank's eighth of C4, the reference's two
# benchmark protocols (repeat: the 30^3 chain incl. C1; sweep: the 20 cells), the heavy legs once
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r04c4}; mkdir -p $OUT
bash tools/r04_check.sh ${1:-r04c4} || exit 1
timeout -k 10 200 python tools/c4_eighth.py > $OUT/c4_eighth.json 2> $OUT/c4_eighth.err || { tail -20 $OUT/c4_eighth.err; exit 1; }
cat $OUT/c4_eighth.json
timeout -k 10 300 python tools/bench_protocol.py repeat --repeat-iters 10 > $OUT/protocol_repeat.csv 2> $OUT/protocol.err || { tail -20 $OUT/protocol.err; exit 1; }
cat $OUT/protocol_repeat.csv
timeout -k 10 400 python tools/bench_protocol.py sweep > $OUT/protocol_sweep.csv 2>> $OUT/protocol.err || { tail -20 $OUT/protocol.err; exit 1; }
tail -3 $OUT/protocol_sweep.csv
timeout -k 10 400 python tools/ab_heavy.py --reps 1 --big tree > $OUT/heavy.txt 2>&1 || { tail -20 $OUT/heavy.txt; exit 1; }
cat $OUT/heavy.txt
