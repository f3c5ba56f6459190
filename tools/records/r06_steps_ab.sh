#!/bin/bash
# round 6: what separates the driver's 20-step line from the 200-step one (timed-step share, warm-up)
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
run() {  # tag, args...
  local t=$1; shift
  timeout -k 10 120 python3 bench.py --gpus 1 --no-cpu --e2e-steps 0 --no-c4 "$@" > gpurun_out/r06_st_$t.json 2> gpurun_out/r06_st_$t.err
  python3 -c "import json;d=json.load(open('gpurun_out/r06_st_$t.json'));print('$t',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'])"
}
for i in 1 2; do
  run s20w5_t10_$i --steps 20 --warmup 5
  run s20w5_t1000_$i --steps 20 --warmup 5 --timing-every 1000
  run s20w50_t10_$i --steps 20 --warmup 50
  run s200w5_t10_$i --steps 200 --warmup 5
  run s200w5_t1000_$i --steps 200 --warmup 5 --timing-every 1000
done
