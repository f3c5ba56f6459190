#!/bin/bash
# Round-4 profiles, second box: C4's kernel trace and FETCH / WRITE / SQ passes, the heavy products'
# FETCH / WRITE / SQ passes (R-MAT 2^16 A^2, C5 2^16 any order), then the multi-rank path on one GPU
# (dist tests, RCCL at world size 1 with the collective path forced, 2 gloo ranks sharing the GPU).
# Every counter group in a pass of its own, each step under its own limit.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r04fb}; mkdir -p $OUT
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/c4trace -o c4 --output-format csv -- python3 tools/prof_c4.py > $OUT/c4trace.log 2>&1 || { tail $OUT/c4trace.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/c4pmc1 -o c4 --output-format csv -- python3 tools/prof_c4.py > $OUT/c4pmc1.log 2>&1 || { tail $OUT/c4pmc1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/c4pmc2 -o c4 --output-format csv -- python3 tools/prof_c4.py > $OUT/c4pmc2.log 2>&1 || { tail $OUT/c4pmc2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS -d $OUT/c4pmc3 -o c4 --output-format csv -- python3 tools/prof_c4.py > $OUT/c4pmc3.log 2>&1 || { tail $OUT/c4pmc3.log; exit 1; }
python3 tools/pmc_summary.py "$OUT/c4pmc*/**/*counter_collection.csv" > $OUT/c4_pmc.json && head -c 1500 $OUT/c4_pmc.json
bash tools/r04_heavy_pmc.sh ${1:-r04fb}/heavy || exit 1
timeout -k 10 300 python -u -m pytest tests/test_dist_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/dist_pytest.log 2>&1 || { tail -40 $OUT/dist_pytest.log; exit 1; }
tail -2 $OUT/dist_pytest.log
timeout -k 10 200 python tools/c4_eighth.py > $OUT/c4_eighth.json 2> $OUT/c4_eighth.err || { tail -20 $OUT/c4_eighth.err; exit 1; }
cat $OUT/c4_eighth.json
SLAT_FORCE_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --e2e-steps 0 > $OUT/strong1.json 2> $OUT/strong1.err || { tail -30 $OUT/strong1.err; exit 1; }
cat $OUT/strong1.json
SLAT_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu --e2e-steps 0 > $OUT/gloo2.json 2> $OUT/gloo2.err || { tail -30 $OUT/gloo2.err; exit 1; }
cat $OUT/gloo2.json
