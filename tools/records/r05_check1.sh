#!/bin/bash
# GPU suite on the round-5 tree, e2e probe, C4 whole vs eighth trace, numeric_short phase counters
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r05c1}; mkdir -p $OUT
if [ -z "$NOTEST" ]; then
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
fi
timeout -k 10 120 python3 tools/c4_eighth.py > $OUT/c4_eighth.json 2>&1 || { tail $OUT/c4_eighth.json; exit 1; }
cat $OUT/c4_eighth.json
SLAT_LIB_PATH=tools/var/libslat_base4.so timeout -k 10 120 python3 tools/c4_eighth.py > $OUT/c4_eighth_base4.json 2>&1 || { tail $OUT/c4_eighth_base4.json; exit 1; }
cat $OUT/c4_eighth_base4.json
timeout -k 10 300 python3 tools/ab_heavy.py --big --reps 1 --legs c5ord,c5big_ord,c5any,c5big_any tree base4 > $OUT/heavy.txt 2>&1 || { tail $OUT/heavy.txt; exit 1; }
tail -6 $OUT/heavy.txt
SLAT_LIB_PATH=tools/var/libslat_knobs.so SLAT_HOSTIO_CLOCK=1 timeout -k 10 120 python3 tools/e2e_ab.py > $OUT/e2e.jsonl 2> $OUT/e2e.err || exit 1
cat $OUT/e2e.jsonl; tail -3 $OUT/e2e.err
timeout -k 10 60 python3 - <<'PY'
import numpy as np, time
for rep in range(3):
    t=time.perf_counter(); a=np.empty(47_000_000//4*4, np.uint32); t1=time.perf_counter(); a[::1024]=0; t2=time.perf_counter(); a[:]=1; t3=time.perf_counter()
    print(f"alloc {1e3*(t1-t):.3f} ms, touch {1e3*(t2-t1):.3f} ms, fill {1e3*(t3-t2):.3f} ms")
PY
cat /sys/kernel/mm/transparent_hugepage/enabled 2>&1
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/trace -o c4e --output-format csv -- python3 tools/prof_c4_eighth.py > $OUT/trace.log 2>&1 || { tail $OUT/trace.log; exit 1; }
grep "C4" $OUT/trace.log
SLAT_LIB_PATH=tools/var/libslat_phases.so timeout -k 10 120 python3 tools/prof_c4_eighth.py > $OUT/phases.log 2>&1 || { tail $OUT/phases.log; exit 1; }
grep -v "^$" $OUT/phases.log | tail -30
