#!/bin/bash
# A/B of the cfg5 notary commit over library variants (CORDAHIP_LIB paths; "-" = in-tree build)
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/${TAG:-abuniq}
mkdir -p $OUT
cd $REPO
for v in "$@"; do
  lib=""; [ "$v" != "-" ] && lib="$REPO/$v"
  CORDAHIP_LIB=$lib timeout -k 10 300 python3 bench.py --sigs 65536 --cold-n 0 --no-txid --no-ecdsa --no-cpu-baseline --no-host-path --no-notary-check > $OUT/b.json 2>>$OUT/err.log || { echo "variant $v failed"; tail -5 $OUT/err.log; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b.json')); s=d['secondary']; print('$v', round(s['notary_commit_ms'],4), round(s['notary_roofline']['frac'],4))" | tee -a $OUT/ab.txt
done
