#!/bin/bash
# tree library vs tools/bin/libslat_$1.so: the GPU parity suite on the tree, then bench.py alternated
set -o pipefail
OUT=gpurun_out/ab_lib; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -n 30 $OUT/tests.log; exit 1; }
tail -n 1 $OUT/tests.log
for i in 1 2; do
  for v in $1 tree; do
    if [ $v = tree ]; then unset SLAT_LIB_PATH; else export SLAT_LIB_PATH=tools/bin/libslat_$v.so; fi
    timeout -k 10 90 python bench.py --no-cpu --steps 300 --warmup 50 > $OUT/$v$i.json 2> $OUT/$v$i.err || { tail $OUT/$v$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/$v$i.json'));print('$v$i', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done
