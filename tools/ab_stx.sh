#!/bin/bash
# A/B of the Kryo front end (tools/bench_stx.py) over library variants ("-" = the in-tree build).
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/${TAG:-abstx}
mkdir -p $OUT
cd $REPO
for v in "$@"; do
  lib=""; [ "$v" != "-" ] && lib="$REPO/$v"
  CORDAHIP_LIB=$lib timeout -k 10 200 python3 tools/bench_stx.py --steps ${STEPS:-5} > $OUT/b.json 2>>$OUT/err.log || { echo "variant $v failed"; tail -5 $OUT/err.log; exit 1; }
  echo "$v $(cat $OUT/b.json)" | tee -a $OUT/ab.txt
done
