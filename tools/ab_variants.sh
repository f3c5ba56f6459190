#!/bin/bash
# bench A/B across library builds (tree | nofused | a tools/bin/libslat_NAME.so variant): ms/step, kernel split
set -o pipefail
OUT=gpurun_out/${1:-fab}; shift
mkdir -p $OUT
export TMPDIR=/tmp
for v in "$@"; do
  if [ $v = nofused ]; then export SLAT_NO_FUSED=1; unset SLAT_LIB_PATH; elif [ $v = tree ]; then unset SLAT_NO_FUSED SLAT_LIB_PATH; else unset SLAT_NO_FUSED; export SLAT_LIB_PATH=tools/bin/libslat_$v.so; fi
  timeout -k 10 60 python bench.py --no-cpu --steps 100 --warmup 30 > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/b.json'));print('$v', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
done
