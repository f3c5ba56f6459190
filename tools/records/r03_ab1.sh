#!/bin/bash
# Round-3 A/B 1: short-row register caps (C4), next-row prefetch in numeric / symbolic (headline),
# the waves_per_eu(4) variant's tests once, and the k_numeric phase split of the headline
set -o pipefail
OUT=gpurun_out/r03b; mkdir -p $OUT
timeout -k 10 900 python tools/ab.py --reps 2 --c4 tree short5 short4 pre1 pre2 spre p1s p2s > $OUT/ab.txt 2>&1 || { tail -30 $OUT/ab.txt; exit 1; }
cat $OUT/ab.txt
SLAT_LIB_PATH=tools/var/libslat_phases.so timeout -k 10 120 python tools/ab.py --child --steps 40 > $OUT/phases.json 2> $OUT/phases.txt || { tail -30 $OUT/phases.txt; exit 1; }
tail -n 2 $OUT/phases.txt
SLAT_LIB_PATH=tools/var/libslat_phases.so timeout -k 10 120 python tools/ab.py --child --only-c4 --steps 100 > $OUT/phases_c4.json 2> $OUT/phases_c4.txt || { tail -30 $OUT/phases_c4.txt; exit 1; }
tail -n 2 $OUT/phases_c4.txt
SLAT_LIB_PATH=tools/var/libslat_wpe4.so timeout -k 10 300 python -u -m pytest tests/test_spgemm_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/wpe4_tests.log 2>&1 || { tail -30 $OUT/wpe4_tests.log; exit 1; }
tail -n 2 $OUT/wpe4_tests.log
SLAT_LIB_PATH=tools/var/libslat_wpe4.so timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu --no-c4 > $OUT/wpe4_bench.json 2> $OUT/wpe4_bench.err || { tail -30 $OUT/wpe4_bench.err; exit 1; }
cat $OUT/wpe4_bench.json
bash tools/r03_heavy.sh
