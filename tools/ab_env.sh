#!/bin/bash
# A/B of tools/bench_ecdsa.py (cfg3 leg) under environment variants given as arguments
# ("VAR=1 VAR2=0" per argument; "-" = defaults).  One JSON line per variant.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/${TAG:-abenv}
mkdir -p $OUT
cd $REPO
for v in "$@"; do
  [ "$v" = "-" ] && v=""
  echo "== $v" >> $OUT/ab.jsonl
  env $v timeout -k 10 120 python3 tools/bench_ecdsa.py --steps 5 >> $OUT/ab.jsonl 2>>$OUT/ab.err || { echo "variant '$v' failed"; tail -5 $OUT/ab.err; exit 1; }
done
cat $OUT/ab.jsonl
