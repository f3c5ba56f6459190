#!/bin/bash
# one-block scan (k_scan_small) for n <= 32768: spgemm / stored / prepared / dist tests on the tree,
# the spgemm tests again on a variant whose two-scan and reload paths run for small counts, then the
# headline + chain A/B against the committed build
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r06scan}; mkdir -p $OUT
T="tests/test_spgemm_gpu.py tests/test_stored_mode_gpu.py tests/test_prepared_gpu.py tests/test_dist_hip_gpu.py tests/test_tiny_gpu.py"
timeout -k 10 600 python -u -m pytest $T -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -v "^  File\|^    " $OUT/pytest.log | tail -30; exit 1; }
tail -n 2 $OUT/pytest.log
SLAT_LIB_PATH=tools/var/libslat_split.so timeout -k 10 600 python -u -m pytest tests/test_spgemm_gpu.py tests/test_stored_mode_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_split.log 2>&1 || { grep -v "^  File\|^    " $OUT/pytest_split.log | tail -30; exit 1; }
tail -n 2 $OUT/pytest_split.log
timeout -k 10 500 python3 tools/ab.py --reps 3 --chain tree base > $OUT/ab.txt 2>&1 || { tail $OUT/ab.txt; exit 1; }
tail -n 3 $OUT/ab.txt
