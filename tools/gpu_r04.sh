#!/bin/bash
# Round-4 GPU check: the VALU issue table (microbench_valu), every -m gpu test, smoke(), the default bench.
#   tools/gpu_r04.sh <tag> [mb|tests|all]
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/${1:-r04}
mkdir -p $OUT
cd $REPO
WHAT=${2:-all}
if [ "$WHAT" = "mb" ] || [ "$WHAT" = "all" ]; then
  timeout -k 10 240 ./tools/microbench_valu > $OUT/microbench_valu.txt 2>&1 || { echo "microbench failed"; tail -20 $OUT/microbench_valu.txt; exit 1; }
  cat $OUT/microbench_valu.txt
fi
[ "$WHAT" = "mb" ] && exit 0
timeout -k 10 700 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
[ "$WHAT" = "tests" ] && exit 0
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
tail -c 600 $OUT/bench.json
