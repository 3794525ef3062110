#!/bin/bash
# per-kernel times of the Kryo front end at 1M blobs (tools/bench_stx.py under rocprofv3 --kernel-trace --stats)
set -uo pipefail
TAG=${1:-kryo_prof}
mkdir -p gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_stx.py --steps 5 > $GRAFT_REPO_ROOT/gpurun_out/$TAG/b.json 2> $GRAFT_REPO_ROOT/gpurun_out/$TAG/err.log || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/$TAG/err.log; exit 1; }
f=$(find $GRAFT_REPO_ROOT/gpurun_out/$TAG/prof -name '*kernel_stats.csv' | head -1)
cp "$f" $GRAFT_REPO_ROOT/gpurun_out/$TAG/kernel_stats.csv
cut -d, -f1-5 $GRAFT_REPO_ROOT/gpurun_out/$TAG/kernel_stats.csv | head -25
