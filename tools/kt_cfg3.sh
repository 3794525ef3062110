#!/bin/bash
# Kernel trace of the cfg3 (ECDSA) leg alone (bench.py with a small cfg2 batch and no other legs) -> gpurun_out/<TAG>/kt
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/${TAG:-ktcfg3}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 $REPO/bench.py --steps 5 --sigs 65536 --cold-n 0 --no-txid --no-notary --no-cpu-baseline --no-host-path --no-key-cache --no-group --no-full-oracle ${EXTRA:-} > $OUT/b.json 2> $OUT/b.err || { echo "trace failed"; tail -5 $OUT/b.err; exit 1; }
