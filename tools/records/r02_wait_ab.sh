#!/bin/bash
# end-of-call wait A/B: k_signal (default) vs hipStreamWriteValue64 (SLAT_WAIT=write), alternated
set -o pipefail
OUT=gpurun_out/wait_ab; mkdir -p $OUT
timeout -k 10 120 python -u -m pytest tests/test_spgemm_gpu.py -x -q --timeout 60 --timeout-method thread > $OUT/tests_default.log 2>&1 || { tail -n 20 $OUT/tests_default.log; exit 1; }
SLAT_WAIT=write timeout -k 10 120 python -u -m pytest tests/test_spgemm_gpu.py tests/test_graph_gpu.py -x -q --timeout 60 --timeout-method thread > $OUT/tests_write.log 2>&1 || { tail -n 20 $OUT/tests_write.log; exit 1; }
tail -n 1 $OUT/tests_default.log $OUT/tests_write.log
for i in 1 2; do
  for m in signal write; do
    if [ $m = write ]; then export SLAT_WAIT=write; else unset SLAT_WAIT; fi
    timeout -k 10 90 python bench.py --no-cpu --steps 300 --warmup 50 > $OUT/$m$i.json 2> $OUT/$m$i.err || { tail $OUT/$m$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/$m$i.json'));print('$m$i', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done
