#!/bin/bash
# Round-3 call ac: RowWalker tail compaction with a round's permutes issued together (variant tb):
# targeted tests, A/B on the headline / C4 / Sat64; the default bench line twice (box spread)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03ac; mkdir -p $OUT
SLAT_LIB_PATH=tools/var/libslat_tb.so timeout -k 10 400 python -u -m pytest tests/test_spgemm_gpu.py tests/test_wide_hash_gpu.py tests/test_graph_gpu.py tests/test_magnus_usize_gpu.py tests/test_real_graph_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests_tb.log 2>&1 || { tail -40 $OUT/tests_tb.log; exit 1; }
tail -n 1 $OUT/tests_tb.log
timeout -k 10 900 python tools/ab.py --reps 4 --c4 --sat64 tree tb > $OUT/ab.txt 2>&1 || { tail -30 $OUT/ab.txt; exit 1; }
grep -A3 summary $OUT/ab.txt
for i in 1 2; do
timeout -k 10 240 python bench.py --no-cpu > $OUT/bench$i.json 2> $OUT/bench$i.err || { tail -20 $OUT/bench$i.err; exit 1; }
python3 -c "import json;d=json.loads(open('$OUT/bench$i.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
done
echo done
