#!/bin/bash
# A/B of the cfg3 (ECDSA) leg over library variants ("-" = the in-tree build), one line per variant
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/${TAG:-abec}
mkdir -p $OUT
cd $REPO
for v in "$@"; do
  lib=""; [ "$v" != "-" ] && lib="$REPO/$v"
  CORDAHIP_LIB=$lib timeout -k 10 300 python3 bench.py --steps ${STEPS:-10} --sigs 65536 --cold-n 0 --no-txid --no-notary --no-cpu-baseline --no-host-path --no-key-cache --no-group --no-full-oracle > $OUT/b.json 2>>$OUT/err.log || { echo "variant $v failed"; tail -5 $OUT/err.log; exit 1; }
  python3 -c "import json; s=json.load(open('$OUT/b.json'))['secondary']; print('$v', round(s['ecdsa_mixed_sigs_per_s']/1e6,2), 'M/s', 'front', round(s['ecdsa_front_ms'],3), 'q', round(s['ecdsa_q_kernel_ms'],3), 'ok', s['ecdsa_correct_vs_labels'])" | tee -a $OUT/ab.txt
done
