#!/bin/bash
# A/B of the cold-key leg (200k Ed25519 signatures, one key each) under environment variants given as arguments
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-abc}; shift
OUT=$REPO/gpurun_out/$TAG
mkdir -p $OUT
cd $REPO
for v in "$@"; do
  env $v timeout -k 10 200 python3 bench.py --sigs 65536 --steps 5 --no-key-cache --no-host-path --no-txid --no-ecdsa --no-notary --no-group --no-cpu-baseline --no-full-oracle > $OUT/b.json 2>>$OUT/err.log || { echo "variant $v failed"; tail -5 $OUT/err.log; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b.json')); s=d['secondary']; print('$v', round(s['ed25519_cold_sigs_per_s']/1e6,2), 'M', s['ed25519_cold_correct'], 'straus', round(s['ed25519_cold_straus_ms'],3), 'keyprep', round(s['ed25519_cold_keyprep_ms'],3))" | tee -a $OUT/ab.txt
done
