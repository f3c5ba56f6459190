#!/bin/bash
# Round-3 A/B 2: held B columns in k_numeric (tree: on; nohold = the round-2 stored bitmaps; hold3 =
# held at 3 waves/SIMD with spills), entries 4-per-lane (segt), u32 parity tests of the tree first
set -o pipefail
OUT=gpurun_out/r03c; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_spgemm_gpu.py tests/test_wide_hash_gpu.py tests/test_short_sort_gpu.py tests/test_graph_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -n 2 $OUT/tests.log
timeout -k 10 900 python tools/ab.py --reps 2 --c4 tree nohold hold3 segt holdsegt > $OUT/ab.txt 2>&1 || { tail -30 $OUT/ab.txt; exit 1; }
cat $OUT/ab.txt
