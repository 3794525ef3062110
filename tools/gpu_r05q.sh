#!/bin/bash
# round 5: cfg4-from-bytes pipeline — the parse stream at a higher priority (CORDA_PARSE_PRIORITY=-1) vs equal
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/${1:-r05q}; mkdir -p $OUT
cd $REPO
for round in 1 2; do
  for v in -1 0; do
    CORDA_PARSE_PRIORITY=$v timeout -k 10 400 python3 bench.py --steps 5 --no-ecdsa --no-notary --cold-n 0 --no-cpu-baseline --no-key-cache --no-host-path --no-full-oracle > $OUT/b_${v}_$round.json 2> $OUT/b.err || { echo "bench $v failed"; tail -5 $OUT/b.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$OUT/b_${v}_$round.json')); s=d['secondary']
print('parse_prio=$v round $round bytes', round(s['cfg4_from_bytes_verified_tx_per_s']/1e6,2), 'M', round(s['cfg4_from_bytes_ms_per_batch'],3), 'ms serial', round(s['cfg4_from_bytes_serial_verified_tx_per_s']/1e6,2), s['cfg4_from_bytes_correct'], 'cfg4', round(s['cfg4_verified_tx_per_s']/1e6,2))" | tee -a $OUT/ab.txt
  done
done
