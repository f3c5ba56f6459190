#!/bin/bash
# round-5 records: the whole GPU suite, the heavy legs (2^16 and 2^18) once each, C4 whole vs eighths
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r05rec}; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python3 tools/ab_heavy.py --child --legs rg,c5any,c5ord,chain > $OUT/heavy16.txt 2>&1 || { tail $OUT/heavy16.txt; exit 1; }
tail -1 $OUT/heavy16.txt | cut -c1-600
timeout -k 10 400 python3 tools/ab_heavy.py --child --big --legs c5big_any,c5big_ord > $OUT/heavy18.txt 2>&1 || { tail $OUT/heavy18.txt; exit 1; }
tail -1 $OUT/heavy18.txt | cut -c1-600
timeout -k 10 120 python3 tools/c4_eighth.py > $OUT/c4_eighth.json 2>&1 || { tail $OUT/c4_eighth.json; exit 1; }
cat $OUT/c4_eighth.json
