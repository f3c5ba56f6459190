#!/bin/bash
# Round-3 profiles: parity tests, smoke, the default bench line, the headline's rocprofv3 trace and
# FETCH/WRITE passes (tools/prof_pmc.sh), C4's trace + FETCH / WRITE / SQ passes, the Sat64 A^6*A
# trace, and the fat-row split table's FETCH_SIZE on C5 2^18 any order (tree vs SLAT_NO_FAT_SPLIT=1).
# Every counter group in a pass of its own.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03j; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -n 2 $OUT/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
timeout -k 10 600 python tools/ab.py --reps 2 --c4 --sat64 tree > $OUT/ab.txt 2>&1 || { tail -30 $OUT/ab.txt; exit 1; }
grep -A3 summary $OUT/ab.txt
SLAT_HOST_CLOCK=1 timeout -k 10 300 python tools/host_overhead.py > $OUT/host.txt 2>&1 || { tail -30 $OUT/host.txt; exit 1; }
tail -4 $OUT/host.txt
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
bash tools/prof_pmc.sh $OUT/prof "--steps 20 --warmup 50 --no-c4" FETCH_SIZE WRITE_SIZE || exit 1
python3 tools/pmc_summary.py $OUT/prof/pmc1/*counter_collection.csv $OUT/prof/pmc2/*counter_collection.csv > $OUT/pmc_summary.json
python3 tools/prof_summary.py $OUT/prof/trace 20 $OUT/pmc_summary.json > $OUT/prof_summary.md && head -12 $OUT/prof_summary.md
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/c4trace -o c4 --output-format csv -- python3 tools/prof_c4.py > $OUT/c4trace.log 2>&1 || { tail $OUT/c4trace.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/c4pmc1 -o c4 --output-format csv -- python3 tools/prof_c4.py > $OUT/c4pmc1.log 2>&1 || { tail $OUT/c4pmc1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/c4pmc2 -o c4 --output-format csv -- python3 tools/prof_c4.py > $OUT/c4pmc2.log 2>&1 || { tail $OUT/c4pmc2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS -d $OUT/c4pmc3 -o c4 --output-format csv -- python3 tools/prof_c4.py > $OUT/c4pmc3.log 2>&1 || { tail $OUT/c4pmc3.log; exit 1; }
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/s7trace -o s7 --output-format csv -- python3 tools/ab.py --child --sat64 --steps 100 > $OUT/s7trace.log 2>&1 || { tail $OUT/s7trace.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fatpmc -o fat --output-format csv -- python3 tools/ab_heavy.py --child --big --legs c5big_any > $OUT/fatpmc.log 2>&1 || { tail $OUT/fatpmc.log; exit 1; }
SLAT_NO_FAT_SPLIT=1 timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fatpmc_nosplit -o fat --output-format csv -- python3 tools/ab_heavy.py --child --big --legs c5big_any > $OUT/fatpmc_nosplit.log 2>&1 || { tail $OUT/fatpmc_nosplit.log; exit 1; }
echo done
