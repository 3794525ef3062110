#!/bin/bash
# Round-3 GPU check: the Kryo front-end tests first, then every -m gpu test, smoke(), the default bench.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/${1:-r03}
mkdir -p $OUT
cd $REPO
timeout -k 10 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_gpu_stx.py > $OUT/gpu_stx.log 2>&1 || { echo "stx tests failed"; tail -60 $OUT/gpu_stx.log; exit 1; }
tail -1 $OUT/gpu_stx.log
[ "${2:-all}" = "stx" ] && exit 0
timeout -k 10 700 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
tail -c 600 $OUT/bench.json
