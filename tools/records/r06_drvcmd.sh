#!/bin/bash
# round 6: the driver's exact bench command against the builder's default (warm-up sensitivity)
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06_drv_$i.json 2> gpurun_out/r06_drv_$i.err
  python3 -c "import json;d=json.load(open('gpurun_out/r06_drv_$i.json'));print('drv',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'] if 'kernel_ms' in d['roofline'] else '')"
done
timeout -k 10 120 python3 bench.py --gpus 1 --no-cpu --e2e-steps 0 > gpurun_out/r06_def.json 2> gpurun_out/r06_def.err
python3 -c "import json;d=json.load(open('gpurun_out/r06_def.json'));print('def',d['value'],d['ms_per_step'])"
