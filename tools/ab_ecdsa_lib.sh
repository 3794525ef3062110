#!/bin/bash
# A/B of the cfg3 leg (tools/bench_ecdsa.py) over library variants (CORDAHIP_LIB paths; "-" = in-tree)
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/${TAG:-abecl}
mkdir -p $OUT
cd $REPO
for v in "$@"; do
  lib=""; [ "$v" != "-" ] && lib="$REPO/$v"
  echo "== $v" >> $OUT/ab.jsonl
  CORDAHIP_LIB=$lib timeout -k 10 150 python3 tools/bench_ecdsa.py --steps 5 ${EXTRA:-} >> $OUT/ab.jsonl 2>>$OUT/ab.err || { echo "variant $v failed"; tail -5 $OUT/ab.err; exit 1; }
done
cat $OUT/ab.jsonl
