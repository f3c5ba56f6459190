#!/bin/bash
# bitmap passes with a group's same-word bits merged (merge) against one atomic per column (k18)
# and the previous tree (k17); C4's short-row
# tiles of 64 rows (default) against 32 / 16 (SLAT_TILE_ROWS, now also for wide launches); parity first
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r04ab12}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_spgemm_gpu.py -k "lane or golden or single_window or bitmap or torus" -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -n 1 $OUT/pytest.log
timeout -k 10 900 python tools/ab.py --reps 2 --steps 100 --chain --c4 k18 merge lr32 pg4 pg4lr32 k18:SLAT_TILE_ROWS=32 > $OUT/ab.txt 2>&1 || { tail -30 $OUT/ab.txt; exit 1; }
grep -A5 summary $OUT/ab.txt | cut -c1-300
# the cost of the HIP-event steps in bench.py's timed region (every 4th step by default)
for TE in 4 1000 4 1000; do
  timeout -k 10 200 python bench.py --no-cpu --no-c4 --e2e-steps 0 --timing-every $TE > $OUT/bench_te$TE.json 2> $OUT/bench_te$TE.err || { tail -20 $OUT/bench_te$TE.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/bench_te$TE.json')); print('timing-every $TE', d['ms_per_step'], d['value'])"
done
# C4 against one rank's eighth of its rows (the 8-way strong-scaling share) by short-row tile size
L=tools/var/libslat_k18.so
SLAT_LIB_PATH=$L timeout -k 10 200 python tools/c4_eighth.py > $OUT/eighth_def.json 2> $OUT/eighth.err || { tail -20 $OUT/eighth.err; exit 1; }
echo "tile default: $(cat $OUT/eighth_def.json)"
for TR in 32 16 8; do
  SLAT_LIB_PATH=$L SLAT_TILE_ROWS=$TR timeout -k 10 200 python tools/c4_eighth.py > $OUT/eighth_t$TR.json 2> $OUT/eighth.err || { tail -20 $OUT/eighth.err; exit 1; }
  echo "tile $TR: $(cat $OUT/eighth_t$TR.json)"
done
