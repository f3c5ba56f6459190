#!/bin/bash
# Round-2 probe: GPU parity tests, the default bench, the host-overhead split and numeric-pass
# ablations of the current pipeline (the data the round's kernel work starts from).
set -o pipefail
OUT=gpurun_out/${1:-r02_probe}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 200 python bench.py --no-cpu > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 120 python tools/host_overhead.py > $OUT/host.txt 2>&1 || { cat $OUT/host.txt; exit 1; }
cat $OUT/host.txt
for cfg in "SLAT_ABLATE=8" "SLAT_ABLATE=16" "SLAT_ABLATE=24" "SLAT_NO_SBM=1"; do
  tag=$(echo "$cfg" | tr ' =/' '_-+')
  env $cfg timeout -k 10 120 python bench.py --no-cpu --steps 40 --warmup 20 > $OUT/$tag.json 2> $OUT/$tag.err || { tail $OUT/$tag.err; exit 1; }
  python - "$cfg" $OUT/$tag.json <<'EOF'
import json, sys
d = json.loads(open(sys.argv[2]).read())
print(sys.argv[1], d["value"], d["roofline"]["kernel_ms"], d["config"].get("ablated_ms"))
EOF
done
