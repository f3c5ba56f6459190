#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/r04_ab2.sh r04ab2 && bash tools/r04_trace1.sh r04tr1
