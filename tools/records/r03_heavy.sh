#!/bin/bash
# Round-3: kernel trace of the power-law / long-row products (RG R-MAT 2^16 A^2, C5 2^16 f64 both
# orders, a dense chain step), and C5 at 2^18 in both orders, for the long-row category decisions
set -o pipefail
OUT=gpurun_out/r03h; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 tools/prof_heavy.py > $OUT/heavy.txt 2> $OUT/heavy.err || { tail -30 $OUT/heavy.err; exit 1; }
cat $OUT/heavy.txt
find $OUT/trace -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/kernel_stats.csv
head -30 $OUT/kernel_stats.csv
