#!/bin/bash
# Round evidence on one GPU box: every -m gpu test, smoke, then tools/profile.sh (default bench under a
# kernel trace + the PMC passes).  Each step under its own time limit; stop at the first failure.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-round}
OUT=$REPO/gpurun_out/$TAG
mkdir -p $OUT
cd $REPO
timeout -k 10 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
bash tools/profile.sh $TAG || { echo "profile failed"; exit 1; }
