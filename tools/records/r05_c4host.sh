#!/bin/bash
# C4 eighth: host split of a call (SLAT_HOST_CLOCK), and tiles below 8 rows
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r05c4h}; mkdir -p $OUT
timeout -k 10 120 python3 - > $OUT/hostclock.log 2>&1 <<'PY' || { tail $OUT/hostclock.log; exit 1; }
import os, sys
os.environ["SLAT_LIB_PATH"] = "tools/var/libslat_knobs.so"
os.environ["SLAT_HOST_CLOCK"] = "1"
sys.path.insert(0, "sparse-linear-algebra-tests_amd")
import slat
ctx = slat.Context(0)
A = slat.torus_thinned_device(100, 3.0, slat.StdRng(), ctx)
P = A.matmul(A).matmul(A)
B = A.prepare()
n = P.n
for _ in range(64 + 512):
    C = P.matmul_rowblock(0, n // 8, B, 0)
    del C
PY
grep "host us" $OUT/hostclock.log | tail -2
for t in 4 6 8; do
SLAT_LIB_PATH=tools/var/libslat_knobs.so SLAT_TILE_ROWS=$t timeout -k 10 120 python3 tools/c4_eighth.py > $OUT/t$t.json 2>&1 || { tail $OUT/t$t.json; exit 1; }
echo "T=$t $(cat $OUT/t$t.json)"
done
timeout -k 10 120 python3 tools/c4_eighth.py > $OUT/tree.json 2>&1 || { tail $OUT/tree.json; exit 1; }
echo "tree $(cat $OUT/tree.json)"
