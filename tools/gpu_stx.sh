#!/bin/bash
# Kryo front-end check on one GPU box: the stx GPU tests, a cfg2 + cfg4 bench (incl. the from-bytes leg),
# and the same bench under a kernel trace (per-kernel times of the parse passes, scans, key interning).
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-stx}
OUT=$REPO/gpurun_out/$TAG
mkdir -p $OUT
cd $REPO
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_stx.py > $OUT/t.log 2>&1 || { echo "tests failed"; tail -30 $OUT/t.log; exit 1; }
tail -2 $OUT/t.log
ARGS="--steps 3 --warmup 1 --no-ecdsa --no-notary --cold-n 0 --no-cpu-baseline --no-host-path"
timeout -k 10 400 python bench.py $ARGS > $OUT/b.json 2> $OUT/b.err || { echo "bench failed"; tail -20 $OUT/b.err; exit 1; }
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 $REPO/bench.py $ARGS > $OUT/bkt.json 2> $OUT/bkt.err || { echo "kt failed"; tail -20 $OUT/bkt.err; exit 1; }
find $OUT/kt -name "*kernel_stats.csv" | head -3
