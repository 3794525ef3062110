#!/bin/bash
# A/B of the cfg2 headline over library variants: each argument is a CORDAHIP_LIB path ("-" = the
# in-tree build).  One line per variant: sigs/s and the per-kernel device times.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/${TAG:-ablib}
mkdir -p $OUT
cd $REPO
for v in "$@"; do
  lib=""; [ "$v" != "-" ] && lib="$REPO/$v"
  CORDAHIP_LIB=$lib timeout -k 10 200 python3 bench.py --steps ${STEPS:-10} --cold-n 0 --no-txid --no-ecdsa --no-notary --no-cpu-baseline --no-host-path ${EXTRA:-} > $OUT/b.json 2>>$OUT/err.log || { echo "variant $v failed"; tail -5 $OUT/err.log; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b.json')); r=d['roofline']; print('$v', round(d['value']/1e6,2), 'M/s', d['correct_vs_labels'], {k: round(x,3) for k,x in r['pipeline_ms'].items()})" | tee -a $OUT/ab.txt
done
