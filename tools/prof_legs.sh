#!/bin/bash
# Kernel trace + FETCH / WRITE passes over the bench's tx-id, fused and notary legs only (no cfg3, no cold keys,
# no CPU baselines): per-kernel times and bytes for the uniqueness and tx-id kernels.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/${1:-legs}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-host-path --no-notary-check --no-ecdsa --cold-n 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 $REPO/bench.py $ARGS > $OUT/b_kt.json 2> $OUT/b_kt.err || { tail -5 $OUT/b_kt.err; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $c -d $OUT/$c -o $c --output-format csv -- python3 $REPO/bench.py $ARGS > $OUT/b_$c.json 2> $OUT/b_$c.err || { tail -5 $OUT/b_$c.err; exit 1; }
  python3 $REPO/tools/pmc_summary.py $(find $OUT/$c -name "*counter_collection.csv" | head -1) $OUT/pmc_$c.csv
done
python3 $REPO/tools/uniq_timeline.py $(find $OUT/kt -name "kt_kernel_trace.csv" | head -1) > $OUT/uniq_timeline.txt 2>&1 || true
grep -E "uniq|txid|stx" $OUT/pmc_*.csv
