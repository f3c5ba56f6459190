#!/bin/bash
# round 6: the driver's bench command with the C4 leg between the headline's input build and its
# warm-up (default) against after the headline
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in 1 2 3; do
  for m in last first; do
    if [ $m = last ]; then export SLAT_BENCH_C4_LAST=1; else unset SLAT_BENCH_C4_LAST; fi
    timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --e2e-steps 0 > gpurun_out/r06_c4o_$m$i.json 2> gpurun_out/r06_c4o_$m$i.err
    python3 -c "import json;d=json.load(open('gpurun_out/r06_c4o_$m$i.json'));c=d['config'];print('$m',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],c.get('c1_ms_per_call'),c.get('c4_ms_per_step'))"
  done
done
