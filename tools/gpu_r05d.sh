#!/bin/bash
# round 5: every GPU test, then a same-box A/B of the ECDSA key decode position in an early Ed25519 batch
set -uo pipefail
OUT=gpurun_out/${1:-r05d}; mkdir -p $OUT
timeout -k 10 800 python -u -m pytest -x -v --durations=10 --timeout 200 --timeout-method thread -m gpu tests > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
for round in 1 2 3; do
  for v in 0 1; do
    CHIP_ECKEYS_LATE=$v timeout -k 10 200 python bench.py --steps 10 --no-txid --no-ecdsa --no-notary --cold-n 0 --no-host-path --no-cpu-baseline --no-key-cache > $OUT/b_${v}_$round.json 2> $OUT/b_${v}_$round.err || { echo "bench $v failed"; tail -5 $OUT/b_${v}_$round.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$OUT/b_${v}_$round.json')); r=d['roofline']
print('late=$v round $round', round(d['value']/1e6,1), 'M', round(d['ms_per_step'],3), 'ms', d['correct_vs_labels'], 'ahalf', round(r['kernel_ms'],3), 'b', round(r['pipeline_ms']['comb_bhalf'],3), 'tables', round(r['pipeline_ms']['comb_tables_aux_stream'],3))" | tee -a $OUT/ab.txt
  done
done
