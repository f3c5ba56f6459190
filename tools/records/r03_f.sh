#!/bin/bash
# Round-3 call f: ticket-queue work distribution (SLAT_DYN: 1 = short-row tiles, 3 = + k_numeric
# rows, 0 = fixed stride) against grid oversubscription; VALU cross-lane sort steps (swz = LDS swizzles), on the headline / C4 / Sat64 and the
# power-law products; GPU tests first (default build), C4 counter passes last
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03f; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -n 2 $OUT/tests.log
SLAT_DYN=3 timeout -k 10 600 python -u -m pytest tests/test_spgemm_gpu.py tests/test_f64_any_order_gpu.py tests/test_fat_rows_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/tests_dyn3.log 2>&1 || { tail -40 $OUT/tests_dyn3.log; exit 1; }
tail -n 2 $OUT/tests_dyn3.log
timeout -k 10 900 python tools/ab.py --reps 2 --c4 --sat64 tree swz tree:SLAT_DYN=0 tree:SLAT_DYN=3 tree:SLAT_DYN=0,SLAT_NUM_OVER=2 > $OUT/ab.txt 2>&1 || { tail -30 $OUT/ab.txt; exit 1; }
grep -A8 summary $OUT/ab.txt
timeout -k 10 900 python tools/ab_heavy.py --reps 2 tree swz tree:SLAT_DYN=0 tree:SLAT_DYN=3 > $OUT/ab_heavy.txt 2>&1 || { tail -30 $OUT/ab_heavy.txt; exit 1; }
grep -A8 summary $OUT/ab_heavy.txt
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/c4pmc1 -o c4 --output-format csv -- python3 tools/prof_c4.py > $OUT/c4pmc1.log 2>&1 || { tail $OUT/c4pmc1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/c4pmc2 -o c4 --output-format csv -- python3 tools/prof_c4.py > $OUT/c4pmc2.log 2>&1 || { tail $OUT/c4pmc2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS -d $OUT/c4pmc3 -o c4 --output-format csv -- python3 tools/prof_c4.py > $OUT/c4pmc3.log 2>&1 || { tail $OUT/c4pmc3.log; exit 1; }
echo done
