#!/bin/bash
# Round-3 call v: MAGNUS fine-level reordering of the fat rows' products (products bucketed by
# accumulator chunk in HBM, then each chunk accumulated from its bucket: the tree) against the
# per-chunk re-walk over B split by chunk (SLAT_NO_FAT_BUCKETS=1): time on RG / C5 incl. 2^18, and
# HBM bytes (FETCH_SIZE / WRITE_SIZE, one pass each) of the fat-row kernels for both, per leg
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03v; mkdir -p $OUT
timeout -k 10 900 python tools/ab_heavy.py --reps 2 --big tree tree:SLAT_NO_FAT_BUCKETS=1 > $OUT/ab_heavy.txt 2>&1 || { tail -30 $OUT/ab_heavy.txt; exit 1; }
grep -A3 summary $OUT/ab_heavy.txt
for leg in rg c5big_any; do
  for v in bucket rewalk; do
    for C in FETCH_SIZE WRITE_SIZE; do
      if [ $v = rewalk ]; then export SLAT_NO_FAT_BUCKETS=1; else unset SLAT_NO_FAT_BUCKETS; fi
      timeout -s KILL 150 rocprofv3 --pmc $C -d $OUT/pmc_${leg}_${v}_$C -o run --output-format csv -- python3 tools/ab_heavy.py --child --legs $leg > $OUT/pmc_${leg}_${v}_$C.log 2>&1 || { tail -20 $OUT/pmc_${leg}_${v}_$C.log; exit 1; }
    done
  done
done
unset SLAT_NO_FAT_BUCKETS
echo done
