#!/bin/bash
# round-6 records on one box: the GPU suite, the default bench line, the headline's kernel trace and its
# FETCH / WRITE / SQ counter passes (profiles/r06*_pmc_torus30_a7.json for bench.py's roofline.traffic),
# each step under its own time limit
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
TAG=${1:-r06final}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -v "^  File\|^    " $OUT/pytest.log | tail -40; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
tail -c 1500 $OUT/bench.json
SQ="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS"
bash tools/prof_pmc.sh $OUT/head "--steps 20 --warmup 10 --no-c4 --e2e-steps 0" "FETCH_SIZE" "WRITE_SIZE" "$SQ" > $OUT/head.log 2>&1 || { tail $OUT/head.log; exit 1; }
python3 tools/prof_summary.py $OUT/head/trace 20 > $OUT/head_summary.md || exit 1
python3 tools/pmc_headline.py $OUT/head $TAG > $OUT/pmc_torus30_a7.json || exit 1
head -c 800 $OUT/pmc_torus30_a7.json; echo
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/ht -o head --output-format csv -- python3 tools/prof_head.py > $OUT/ht.log 2>&1 || { tail $OUT/ht.log; exit 1; }
grep headline $OUT/ht.log
python3 tools/trace_gaps.py $OUT/ht 12 > $OUT/head_gaps.txt && cat $OUT/head_gaps.txt
