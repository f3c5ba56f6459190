#!/bin/bash
# C4 (or --only X) timing across library builds: tools/ab_suite.sh CELLS lib1 lib2 ... ("tree" = in-tree)
C=$1; shift
for L in "$@"; do
  if [ "$L" = tree ]; then unset SLAT_LIB_PATH; else export SLAT_LIB_PATH=$L; fi
  timeout -k 10 200 python tools/bench_suite.py --only $C --no-cpu --out gpurun_out/abs.json > /dev/null 2>&1 || exit 1
  python3 -c "import json;[print('$L', c['cell'], round(c['gpu_ms'],3), round(c['numeric_ms'],3), round(c['device_ms'],3)) for c in json.load(open('gpurun_out/abs.json'))['cells']]"
done
