#!/bin/bash
# C1 (the lane kernel) phase split (variant build), C1 per call, the pinned e2e split (tree / round 4),
# the GPU suite and a bench line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r05lane3}; mkdir -p $OUT
SLAT_LIB_PATH=tools/var/libslat_phases.so timeout -k 10 120 python3 tools/prof_c1.py > $OUT/phases.out 2> $OUT/phases.log || { tail $OUT/phases.log; exit 1; }
tail -1 $OUT/phases.log
for i in 1 2 3; do timeout -k 10 120 python3 tools/prof_c1.py >> $OUT/c1.out 2>&1 || { tail $OUT/c1.out; exit 1; }; done
cat $OUT/c1.out
for lib in sparse-linear-algebra-tests_amd/libslat.so tools/var/libslat_base4.so sparse-linear-algebra-tests_amd/libslat.so tools/var/libslat_base4.so; do
SLAT_LIB_PATH=$lib timeout -k 10 120 python3 tools/e2e_pinned.py >> $OUT/pin.txt 2>&1 || { tail $OUT/pin.txt; exit 1; }
done
cat $OUT/pin.txt
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 200 python3 bench.py --no-cpu --no-c4 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
cut -c1-300 $OUT/bench.json
