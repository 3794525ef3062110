#!/bin/bash
# A/B runs of the cfg3 leg (tools/bench_ecdsa.py) under environment variants, then one kernel trace.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-ab}
OUT=$REPO/gpurun_out/$TAG
mkdir -p $OUT
cd $REPO
VARS=("")
for v in "${VARS[@]}"; do
  env $v timeout -k 10 120 python3 tools/bench_ecdsa.py --steps 5 >> $OUT/ab.jsonl 2>>$OUT/ab.err || { echo "variant '$v' failed"; tail -5 $OUT/ab.err; exit 1; }
done
timeout -k 10 120 python3 tools/bench_ecdsa.py --steps 5 --p256-only >> $OUT/ab.jsonl 2>>$OUT/ab.err || exit 1
cat $OUT/ab.jsonl
export TMPDIR=/tmp
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/kt -o kt --output-format csv -- python3 $REPO/tools/bench_ecdsa.py --steps 3 > /dev/null 2>$OUT/kt.err || { echo "trace failed"; exit 1; }
