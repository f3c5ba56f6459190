#!/bin/bash
# multi-rank rehearsals on one GPU: torchrun with the RCCL path forced at world size 1, then two gloo
# ranks sharing the GPU (bench.py's N > 1 code: broadcast, device cuts, row blocks, assembly)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r05dist}; mkdir -p $OUT
SLAT_FORCE_DIST=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --e2e-steps 0 > $OUT/rccl1.json 2> $OUT/rccl1.err || { tail -20 $OUT/rccl1.err; exit 1; }
tail -c 900 $OUT/rccl1.json; echo
SLAT_DIST_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu --e2e-steps 0 > $OUT/gloo2.json 2> $OUT/gloo2.err || { tail -20 $OUT/gloo2.err; exit 1; }
tail -c 900 $OUT/gloo2.json; echo
# the lane kernel's compact arguments: its tests, then C1 (chain legs) against the library before
timeout -k 10 300 python -u -m pytest tests/test_spgemm_gpu.py tests/test_dropin_cpp_gpu.py -x -q --timeout 120 --timeout-method thread -k "lane or dropin or torus30" > $OUT/pytest_lane.log 2>&1 || { tail -30 $OUT/pytest_lane.log; exit 1; }
tail -1 $OUT/pytest_lane.log
timeout -k 10 400 python3 tools/ab.py --reps 3 --chain tree base > $OUT/ab.txt 2>&1 || { tail $OUT/ab.txt; exit 1; }
tail -2 $OUT/ab.txt
timeout -k 10 120 python3 tools/host_cabi.py > $OUT/host.txt 2>&1 || { tail $OUT/host.txt; exit 1; }
cat $OUT/host.txt
SLAT_LIB_PATH=tools/var/libslat_base.so timeout -k 10 120 python3 tools/host_cabi.py > $OUT/host_base.txt 2>&1 || { tail $OUT/host_base.txt; exit 1; }
sed 's/^/base /' $OUT/host_base.txt
