#!/bin/bash
# usage: tools/knob_sweep.sh OUT "VAR=val VAR2=val" ["..."]  — one bench.py run per env setting
OUT=$1; shift
mkdir -p $OUT
for cfg in "$@"; do
  tag=$(echo "$cfg" | tr ' =/' '_-+')
  env $cfg timeout -k 10 120 python3 bench.py --no-cpu --steps 10 --warmup 2 > $OUT/$tag.json 2> $OUT/$tag.err || { echo "FAIL $cfg"; exit 1; }
  python3 tools/show_bench.py "$cfg" $OUT/$tag.json
done
