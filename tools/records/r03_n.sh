#!/bin/bash
# Round-3 call n: fat rows with the products bucketed by accumulator chunk (SLAT_NO_FAT_BUCKETS=1:
# one walk per touched chunk) — fat-row tests first, then the heavy A/B; HIP runtime launch knobs on
# the headline (HIP_FORCE_DEV_KERNARG, AMD_DIRECT_DISPATCH)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03n; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_fat_rows_gpu.py tests/test_f64_any_order_gpu.py tests/test_real_graph_gpu.py tests/test_spgemm_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -n 2 $OUT/tests.log
timeout -k 10 1000 python tools/ab_heavy.py --reps 2 --big tree tree:SLAT_NO_FAT_BUCKETS=1 > $OUT/ab_heavy.txt 2>&1 || { tail -30 $OUT/ab_heavy.txt; exit 1; }
grep -A3 summary $OUT/ab_heavy.txt
timeout -k 10 900 python tools/ab.py --reps 2 tree tree:HIP_FORCE_DEV_KERNARG=1 tree:AMD_DIRECT_DISPATCH=0 > $OUT/ab.txt 2>&1 || { tail -30 $OUT/ab.txt; exit 1; }
grep -A4 summary $OUT/ab.txt
echo done
