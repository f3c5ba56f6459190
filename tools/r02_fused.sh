#!/bin/bash
# fused-kernel check: SpGEMM parity tests, then the bench across builds
set -o pipefail
OUT=gpurun_out/${1:-fused}; shift
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_spgemm_gpu.py tests/test_magnus_usize_gpu.py -x -q --timeout 60 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
bash tools/r02_fused_ab.sh $(basename $OUT) "$@"
