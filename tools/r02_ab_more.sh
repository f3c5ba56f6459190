#!/bin/bash
# tree vs tools/bin/libslat_$1.so: bench.py alternated 4 times, then a kernel trace of the tree
set -o pipefail
OUT=gpurun_out/${AB_OUT:-ab_more}; mkdir -p $OUT
for i in 1 2 3 4; do
  for v in $1 tree; do
    if [ $v = tree ]; then unset SLAT_LIB_PATH; else export SLAT_LIB_PATH=tools/bin/libslat_$v.so; fi
    timeout -k 10 90 python bench.py --no-cpu --steps 400 --warmup 50 > $OUT/$v$i.json 2> $OUT/$v$i.err || { tail $OUT/$v$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/$v$i.json'));print('$v$i', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done
unset SLAT_LIB_PATH
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --no-cpu --steps 20 --warmup 50 > $OUT/trace_bench.json 2> $OUT/trace.err || { tail $OUT/trace.err; exit 1; }
python3 tools/prof_summary.py $OUT/trace 20 | head -12
