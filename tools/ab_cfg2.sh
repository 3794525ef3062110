#!/bin/bash
# A/B of the cfg2 headline step (device entry, 1M Ed25519 signatures over 4096 keys) under environment variants given
# as arguments, each variant run twice in alternation (ABAB) on the same box
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-ab2}; shift
OUT=$REPO/gpurun_out/$TAG
mkdir -p $OUT
cd $REPO
for rep in 1 2; do
for v in "$@"; do
  env $v timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 --cold-n 0 --no-key-cache --no-host-path --no-txid --no-ecdsa --no-notary --no-group --no-cpu-baseline --no-full-oracle > $OUT/b.json 2>>$OUT/err.log || { echo "variant $v failed"; tail -5 $OUT/err.log; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b.json')); print('$v', round(d['value']/1e6,2), 'M', round(d['ms_per_step'],4), 'ms', d['correct_vs_labels'])" | tee -a $OUT/ab.txt
done
done
