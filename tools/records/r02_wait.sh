#!/bin/bash
# end-of-call wait A/B on the headline bench (host split from SLAT_HOST_CLOCK)
set -o pipefail
for w in flag sync query flag; do
  SLAT_WAIT=$w SLAT_HOST_CLOCK=1 timeout -k 10 120 python bench.py --no-cpu --steps 512 --warmup 64 > gpurun_out/wait_$w.json 2> gpurun_out/wait_$w.err || { tail gpurun_out/wait_$w.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/wait_$w.json'));print('$w', d['value'], d['ms_per_step'])"
  tail -n 1 gpurun_out/wait_$w.err
done
