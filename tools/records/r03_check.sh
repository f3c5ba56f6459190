#!/bin/bash
# Round-3 GPU check: the GPU suite, the default bench (driver protocol), the RCCL world-1 rehearsal,
# then library variants A/B'd on the headline and C4, and the waves_per_eu(4) variant's tests once
set -o pipefail
OUT=gpurun_out/r03a; mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -n 3 $OUT/tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
SLAT_FORCE_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $OUT/dist1.json 2> $OUT/dist1.err || { tail -30 $OUT/dist1.err; exit 1; }
cat $OUT/dist1.json
timeout -k 10 600 python tools/ab.py --reps 2 --c4 tree short5 short4 > $OUT/ab_short.txt 2>&1 || { tail -30 $OUT/ab_short.txt; exit 1; }
cat $OUT/ab_short.txt
SLAT_LIB_PATH=tools/var/libslat_wpe4.so timeout -k 10 300 python -u -m pytest tests/test_spgemm_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/wpe4_tests.log 2>&1 || { tail -30 $OUT/wpe4_tests.log; exit 1; }
tail -n 2 $OUT/wpe4_tests.log
SLAT_LIB_PATH=tools/var/libslat_wpe4.so timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu --no-c4 > $OUT/wpe4_bench.json 2> $OUT/wpe4_bench.err || { tail -30 $OUT/wpe4_bench.err; exit 1; }
cat $OUT/wpe4_bench.json
