#!/bin/bash
# kernel trace of bench runs with separate (discarded) ablated launches
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for A in "$@"; do
  mkdir -p gpurun_out/tabl/$A
  SLAT_ABLATE=$A timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/tabl/$A -o run --output-format csv -- python3 bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/tabl/$A/bench.json 2> gpurun_out/tabl/$A/err.txt
done
echo ok
