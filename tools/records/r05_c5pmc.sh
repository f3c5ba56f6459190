#!/bin/bash
# C5 2^18 in the fold order after the in-order atomic adds: kernel trace, then FETCH / WRITE / SQ passes
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r05c5pmc}; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o c5 --output-format csv -- python3 tools/ab_heavy.py --child --big --legs c5big_ord > $OUT/c5.log 2>&1 || { tail $OUT/c5.log; exit 1; }
tail -1 $OUT/c5.log | cut -c1-200
python3 tools/trace_table.py $OUT/trace 6
SQ="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS"
i=0; for C in "FETCH_SIZE" "WRITE_SIZE" "$SQ"; do i=$((i+1));
timeout -s KILL 300 rocprofv3 --pmc $C -d $OUT/pmc$i -o c5 --output-format csv -- python3 tools/ab_heavy.py --child --big --legs c5big_ord > $OUT/pmc$i.log 2>&1 || { tail $OUT/pmc$i.log; exit 1; }; done
python3 tools/pmc_summary.py "$OUT/pmc*/**/*counter_collection.csv" > $OUT/c5_pmc.json || exit 1
python3 -c "
import json; d=json.load(open('$OUT/c5_pmc.json'))
for k,v in d.items():
  if 'fr_numeric' in k or 'k_numeric' in k: print(k[:60], {x: v.get(x) for x in ('SQ_INSTS_VALU','SQ_INSTS_LDS','SQ_INSTS_SALU','SQ_WAIT_ANY','SQ_WAVE_CYCLES','SQ_BUSY_CYCLES','hbm_read_bytes_corrected','_dur_ns')})
"
