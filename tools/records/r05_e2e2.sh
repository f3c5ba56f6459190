#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r05e2e3}; mkdir -p $OUT
V=tools/var/libslat_knobs.so
SLAT_LIB_PATH=$V SLAT_HOSTIO_CLOCK=1 timeout -k 10 120 python3 tools/e2e_ab.py > $OUT/e2e.jsonl 2> $OUT/err.log || exit 1
cat $OUT/e2e.jsonl; tail -5 $OUT/err.log
cat /sys/kernel/mm/transparent_hugepage/enabled /sys/kernel/mm/transparent_hugepage/defrag 2>&1
timeout -k 10 60 python3 - <<'PY'
import numpy as np, time
for rep in range(3):
    t=time.perf_counter(); a=np.empty(47_000_000//4*4, np.uint32); t1=time.perf_counter(); a[::1024]=0; t2=time.perf_counter(); a[:]=1; t3=time.perf_counter()
    print(f"alloc {1e3*(t1-t):.3f} ms, touch {1e3*(t2-t1):.3f} ms, fill {1e3*(t3-t2):.3f} ms")
PY
nproc; grep -m1 "model name" /proc/cpuinfo; cat /sys/fs/cgroup/cpu.max 2>/dev/null
