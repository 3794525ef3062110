#!/bin/bash
# A/B of the cfg5 notary leg under environment variants (each variant's line: notary commit ms)
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-abu}; shift
OUT=$REPO/gpurun_out/$TAG
mkdir -p $OUT
cd $REPO
for v in "$@"; do
  env $v timeout -k 10 300 python3 bench.py --sigs 65536 --cold-n 0 --no-txid --no-ecdsa --no-cpu-baseline --no-host-path --no-notary-check --no-group --no-key-cache > $OUT/b.json 2>>$OUT/err.log || { echo "variant $v failed"; tail -5 $OUT/err.log; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b.json')); s=d['secondary']; print('$v', s['notary_commit_ms'], s['notary_roofline']['frac'])" | tee -a $OUT/ab.txt
done
