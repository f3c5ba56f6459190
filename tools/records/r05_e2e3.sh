#!/bin/bash
# e2e: where the pageable call's time goes (library copies vs the caller's page faults / frees)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r05e2e4}; mkdir -p $OUT
cat /proc/cmdline; uname -r; cat /sys/kernel/mm/transparent_hugepage/enabled /sys/kernel/mm/transparent_hugepage/defrag
python3 -c "import numpy as np; print('numpy', np.__version__, 'madvise_hugepage', np.core.multiarray._get_madvise_hugepage() if hasattr(np.core.multiarray,'_get_madvise_hugepage') else '?')"
timeout -k 10 60 python3 - <<'PY'
import numpy as np, time, ctypes, mmap
for rep in range(3):
    t=time.perf_counter(); a=np.empty(47_000_000//4*4, np.uint32); t1=time.perf_counter(); a[::1024]=0; t2=time.perf_counter(); del a; t3=time.perf_counter()
    print(f"np: alloc {1e3*(t1-t):.3f} ms, touch {1e3*(t2-t1):.3f} ms, free {1e3*(t3-t2):.3f} ms")
PY
grep -i -E "AnonHugePages|Hugepagesize" /proc/meminfo
SLAT_LIB_PATH=tools/var/libslat_knobs.so SLAT_HOSTIO_CLOCK=1 timeout -k 10 120 python3 tools/e2e_ab.py > $OUT/e2e.jsonl 2> $OUT/e2e.err || exit 1
GLIBC_TUNABLES=glibc.malloc.mmap_max=0:glibc.malloc.trim_threshold=4294967295 timeout -k 10 120 python3 tools/e2e_ab.py >> $OUT/e2e.jsonl 2>> $OUT/e2e.err || exit 1
cat $OUT/e2e.jsonl; tail -3 $OUT/e2e.err
