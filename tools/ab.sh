#!/bin/bash
# A/B of the bench across library builds, alternating: tools/ab.sh ROUNDS lib1 lib2 ... (path or "tree")
R=$1; shift
for r in $(seq $R); do
  for L in "$@"; do
    if [ "$L" = tree ]; then unset SLAT_LIB_PATH; else export SLAT_LIB_PATH=$L; fi
    timeout -k 10 120 python bench.py --no-cpu --steps 200 --warmup 50 > gpurun_out/ab.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/ab.json'));k=d['roofline']['kernel_ms'];print('$L', d['value'], k['symbolic'], k['numeric'])"
  done
done
