#!/bin/bash
# Quick GPU check of a subset: tests (given as args) then optional bench args via BENCH_ARGS.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-quick}
OUT=$REPO/gpurun_out/$TAG
mkdir -p $OUT
cd $REPO
if [ $# -gt 0 ]; then
  timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread "$@" > $OUT/t.log 2>&1 || { echo "tests failed"; tail -40 $OUT/t.log; exit 1; }
  tail -3 $OUT/t.log
fi
if [ -n "${BENCH_ARGS:-}" ]; then
  timeout -k 10 500 python bench.py $BENCH_ARGS > $OUT/b.json 2> $OUT/b.err || { echo "bench failed"; tail -20 $OUT/b.err; exit 1; }
  tail -c 600 $OUT/b.err
fi
