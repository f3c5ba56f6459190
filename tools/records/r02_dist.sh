#!/bin/bash
# multi-rank path on one GPU: dist GPU tests, the strong bench through torchrun at world size 1 with
# the RCCL code path forced (broadcast, device cuts, allgatherv), and a 2-rank gloo rehearsal
set -o pipefail
OUT=gpurun_out/${1:-dist}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_dist_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
SLAT_FORCE_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $OUT/strong1.json 2> $OUT/strong1.err || { tail -30 $OUT/strong1.err; exit 1; }
cat $OUT/strong1.json
SLAT_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu > $OUT/gloo2.json 2> $OUT/gloo2.err || { tail -30 $OUT/gloo2.err; exit 1; }
cat $OUT/gloo2.json
