#!/bin/bash
# uniqueness GPU tests, then the notary / tx-id legs under the profiler (tools/prof_legs.sh)
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/${1:-uniq}
mkdir -p $OUT
cd $REPO
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_uniq.py tests/test_gpu_cfg1_cash.py > $OUT/tests.log 2>&1 || { echo "uniq tests failed"; tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
bash tools/prof_legs.sh ${1:-uniq}/legs
