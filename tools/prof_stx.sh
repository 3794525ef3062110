#!/bin/bash
# Kryo front end under a kernel + memory-copy trace (tools/bench_stx.py), one parse per step.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/${1:-stx}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $OUT/kt -o kt --output-format csv -- \
    python3 $REPO/tools/bench_stx.py --steps 3 ${2:-} > $OUT/bench_stx.json 2> $OUT/bench_stx.err || { tail -20 $OUT/bench_stx.err; exit 1; }
cat $OUT/bench_stx.json
KT=$(find $OUT/kt -name "kt_kernel_trace.csv" | head -1)
python3 $REPO/tools/kt_timeline.py $OUT/kt --count 70 > $OUT/timeline.txt || true
cat $OUT/timeline.txt
