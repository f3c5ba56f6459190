#!/bin/bash
# per-call host cost (mirror vs C ABI), the C1 kernel trace, a bench line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r05_host}; mkdir -p $OUT
timeout -k 10 120 python3 tools/host_cabi.py > $OUT/host.txt 2>&1 || { tail $OUT/host.txt; exit 1; }
cat $OUT/host.txt
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/c1 -o c1 --output-format csv -- python3 tools/prof_c1.py > $OUT/c1.log 2>&1 || { tail $OUT/c1.log; exit 1; }
grep C1 $OUT/c1.log; grep k_lane $OUT/c1/*/c1_kernel_stats.csv $OUT/c1/c1_kernel_stats.csv 2>/dev/null | cut -c1-160
timeout -k 10 200 python3 bench.py --no-cpu > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
python3 -c "
import json,sys; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); c=d['config']
print({k: d[k] for k in ('value','ms_per_step','scaling_value')}); print({k: c.get(k) for k in ('c1_ms_per_call','c4_ms_per_step','e2e_ms','e2e_heap_ms')})"
