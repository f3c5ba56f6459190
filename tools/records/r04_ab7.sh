#!/bin/bash
# the fold order's fat walk with the next groups' loads in flight (k9) against k8; the host split of
# a call (SLAT_HOST_CLOCK=1)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r04ab7}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_fat_rows_gpu.py tests/test_f64_any_order_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -n 2 $OUT/pytest.log
timeout -k 10 900 python tools/ab_heavy.py --reps 2 --big --legs c5ord,c5big_ord k8 k9 > $OUT/heavy.txt 2>&1 || { tail -30 $OUT/heavy.txt; exit 1; }
tail -n 3 $OUT/heavy.txt | cut -c1-900
SLAT_LIB_PATH=$GRAFT_REPO_ROOT/tools/var/libslat_k9.so SLAT_HOST_CLOCK=1 timeout -k 10 300 python tools/host_overhead.py > $OUT/host.txt 2>&1 || { tail -30 $OUT/host.txt; exit 1; }
tail -6 $OUT/host.txt
