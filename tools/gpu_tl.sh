#!/bin/bash
# kernel timeline of the cfg2 step (kernel trace only)
set -uo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-tl}; mkdir -p $OUT
cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/kt -o kt --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-host-path --no-key-cache --cold-n 0 --no-txid --no-ecdsa --no-notary > $OUT/b.json 2> $OUT/b.err || { echo "trace failed"; tail -5 $OUT/b.err; exit 1; }
python3 $GRAFT_REPO_ROOT/tools/timeline.py $(find $OUT/kt -name "*kernel_trace.csv" | head -1) | tee $OUT/timeline.txt
