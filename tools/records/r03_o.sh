#!/bin/bash
# Round-3 call o: RowWalker segment interleave (variant ilv: lane l holds entries 4l..4l+3, so one
# LDS instruction's lanes hold columns 4 apart) A/B on the headline / C4 / Sat64; then a host-trap PC
# sampling pass over C4 (k_symbolic_short / k_numeric_short instruction hot spots)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03o; mkdir -p $OUT
SLAT_LIB_PATH=tools/var/libslat_ilv.so timeout -k 10 300 python -u -m pytest tests/test_spgemm_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests_ilv.log 2>&1 || { tail -40 $OUT/tests_ilv.log; exit 1; }
tail -n 2 $OUT/tests_ilv.log
timeout -k 10 900 python tools/ab.py --reps 3 --c4 --sat64 tree ilv > $OUT/ab.txt 2>&1 || { tail -30 $OUT/ab.txt; exit 1; }
grep -A3 summary $OUT/ab.txt
timeout -s KILL 180 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 1 -d $OUT/pcs -o c4 --output-format csv -- python3 tools/prof_c4.py > $OUT/pcs.log 2>&1 || { tail -30 $OUT/pcs.log; exit 1; }
tail -3 $OUT/pcs.log
find $OUT/pcs -type f | head -20
echo done1
timeout -s KILL 180 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 1 -d $OUT/pcs_a7 -o a7 --output-format csv -- python3 tools/ab.py --child --steps 400 > $OUT/pcs_a7.log 2>&1 || { tail -30 $OUT/pcs_a7.log; exit 1; }
tail -3 $OUT/pcs_a7.log
echo done2
