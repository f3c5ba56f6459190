#!/bin/bash
# e2e A/B: the staging ring (default library) against the runtime's pageable copies and hipHostRegister
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r05e2e}; mkdir -p $OUT
V=tools/var/libslat_knobs.so
for i in 1 2; do
timeout -k 10 120 python3 tools/e2e_ab.py >> $OUT/e2e.jsonl 2>> $OUT/err.log || exit 1
SLAT_LIB_PATH=$V SLAT_HOSTIO=runtime timeout -k 10 120 python3 tools/e2e_ab.py >> $OUT/e2e.jsonl 2>> $OUT/err.log || exit 1
SLAT_LIB_PATH=$V SLAT_HOSTIO=register timeout -k 10 120 python3 tools/e2e_ab.py >> $OUT/e2e.jsonl 2>> $OUT/err.log || exit 1
SLAT_HOST_THREADS=4 timeout -k 10 120 python3 tools/e2e_ab.py >> $OUT/e2e.jsonl 2>> $OUT/err.log || exit 1
SLAT_HOST_THREADS=16 timeout -k 10 120 python3 tools/e2e_ab.py >> $OUT/e2e.jsonl 2>> $OUT/err.log || exit 1
done
cat $OUT/e2e.jsonl
