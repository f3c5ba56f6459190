#!/bin/bash
# the GPU suite and a bench line (C4 leg and e2e legs included)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r05suite}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python3 bench.py --no-cpu > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
python3 - $OUT/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c = d["config"]
print({k: d[k] for k in ("value", "ms_per_step", "scaling_value")})
print({k: c.get(k) for k in ("c1_ms_per_call", "c1_gnnz_per_s", "c4_ms_per_step", "e2e_ms", "e2e_pinned_ms", "e2e_heap_ms")})
PY
