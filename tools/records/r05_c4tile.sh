#!/bin/bash
# C4 whole vs eighth (prepared B) on the tree, then the tile-rows sweep (variant build with knobs)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r05c4t}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_prepared_gpu.py tests/test_wide_hash_gpu.py tests/test_short_sort_gpu.py tests/test_fat_rows_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 120 python3 tools/c4_eighth.py > $OUT/c4_eighth.json 2>&1 || { tail $OUT/c4_eighth.json; exit 1; }
cat $OUT/c4_eighth.json
for t in 8 12 16 24 32 48 64; do
SLAT_LIB_PATH=tools/var/libslat_knobs.so SLAT_TILE_ROWS=$t timeout -k 10 120 python3 tools/c4_eighth.py > $OUT/t$t.json 2>&1 || { tail $OUT/t$t.json; exit 1; }
echo "T=$t $(cat $OUT/t$t.json)"
done
