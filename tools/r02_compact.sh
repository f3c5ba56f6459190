#!/bin/bash
# compacted numeric bitmap A/B: the new GPU test, then bench.py for the tree, the tree with
# SLAT_COMPACT_BLK=0 (whole window in LDS), and the waves-per-EU variants in tools/bin
set -o pipefail
OUT=gpurun_out/compact; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_spgemm_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -n 30 $OUT/tests.log; exit 1; }
tail -n 2 $OUT/tests.log
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 90 python bench.py --no-cpu --steps 200 --warmup 30 > $OUT/$name.json 2> $OUT/$name.err || { tail $OUT/$name.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$name.json'));print('$name', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
}
run tree X=1
run tree_blk0 SLAT_COMPACT_BLK=0
for v in "$@"; do run $v SLAT_LIB_PATH=tools/bin/libslat_$v.so; done
run tree_again X=1
