#!/bin/bash
# Round-6 records (last session): kernel traces and counter passes (each its own rocprofv3 run):
# C4 (whole + one eighth, B prepared), C1 (the lane kernel) and C5 2^18 in the reference's fold order.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r06prof}; mkdir -p $OUT
SQ="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS"
# 2. C4 whole + eighth (B prepared)
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/c4/trace -o c4 --output-format csv -- python3 tools/prof_c4_eighth.py > $OUT/c4.log 2>&1 || { tail $OUT/c4.log; exit 1; }
grep C4 $OUT/c4.log
i=0; for C in "FETCH_SIZE" "WRITE_SIZE" "$SQ"; do i=$((i+1));
timeout -s KILL 180 rocprofv3 --pmc $C -d $OUT/c4/pmc$i -o c4 --output-format csv -- python3 tools/prof_c4.py > $OUT/c4_pmc$i.log 2>&1 || { tail $OUT/c4_pmc$i.log; exit 1; }; done
python3 tools/pmc_summary.py "$OUT/c4/pmc*/**/*counter_collection.csv" > $OUT/c4_pmc.json || exit 1
# 3. C1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/c1/trace -o c1 --output-format csv -- python3 tools/prof_c1.py > $OUT/c1.log 2>&1 || { tail $OUT/c1.log; exit 1; }
grep C1 $OUT/c1.log
i=0; for C in "FETCH_SIZE" "WRITE_SIZE" "$SQ"; do i=$((i+1));
timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/c1/pmc$i -o c1 --output-format csv -- python3 tools/prof_c1.py > $OUT/c1_pmc$i.log 2>&1 || { tail $OUT/c1_pmc$i.log; exit 1; }; done
python3 tools/pmc_summary.py "$OUT/c1/pmc*/**/*counter_collection.csv" > $OUT/c1_pmc.json || exit 1
# 4. C5 2^18 fold order
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/c5/trace -o c5 --output-format csv -- python3 tools/ab_heavy.py --child --big --legs c5big_ord > $OUT/c5.log 2>&1 || { tail $OUT/c5.log; exit 1; }
tail -1 $OUT/c5.log | cut -c1-300
i=0; for C in "FETCH_SIZE" "WRITE_SIZE" "$SQ"; do i=$((i+1));
timeout -s KILL 300 rocprofv3 --pmc $C -d $OUT/c5/pmc$i -o c5 --output-format csv -- python3 tools/ab_heavy.py --child --big --legs c5big_ord > $OUT/c5_pmc$i.log 2>&1 || { tail $OUT/c5_pmc$i.log; exit 1; }; done
python3 tools/pmc_summary.py "$OUT/c5/pmc*/**/*counter_collection.csv" > $OUT/c5_pmc.json || exit 1
echo profiles done
