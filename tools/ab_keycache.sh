#!/bin/bash
# A/B of the cfg2 headline and its key-cache leg (CHIP_FLAG_KEY_CACHE: the per-key state kept across batches) over
# library variants ("-" = the in-tree build)
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/${TAG:-abkc}
mkdir -p $OUT
cd $REPO
for v in "$@"; do
  lib=""; [ "$v" != "-" ] && lib="$REPO/$v"
  CORDAHIP_LIB=$lib timeout -k 10 300 python3 bench.py --steps ${STEPS:-10} --cold-n 0 --no-txid --no-ecdsa --no-notary --no-cpu-baseline --no-host-path --no-group --no-full-oracle > $OUT/b.json 2>>$OUT/err.log || { echo "variant $v failed"; tail -5 $OUT/err.log; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b.json')); s=d['secondary']; print('$v', 'cfg2', round(d['value']/1e6,2), d['correct_vs_labels'], 'key_cache', round(s['cfg2_key_cache_sigs_per_s']/1e6,2), s.get('cfg2_key_cache_correct'))" | tee -a $OUT/ab.txt
done
