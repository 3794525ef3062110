#!/bin/bash
# round 5: group + Ed25519 tests, then same-box A/B of the Ed25519 table split window (CHIP_ED_SPLIT_W) on cfg2
set -uo pipefail
OUT=gpurun_out/${1:-r05c}; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_group.py tests/test_gpu_ed25519.py tests/test_gpu_key_cache.py tests/test_gpu_host_entry.py > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for round in 1 2; do
  for w in 0 22 16 28; do
    CHIP_ED_SPLIT_W=$w timeout -k 10 200 python bench.py --steps 10 --no-txid --no-ecdsa --no-notary --cold-n 0 --no-host-path --no-cpu-baseline --no-key-cache > $OUT/b_${w}_$round.json 2> $OUT/b_${w}_$round.err || { echo "bench $w failed"; tail -5 $OUT/b_${w}_$round.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$OUT/b_${w}_$round.json')); r=d['roofline']
print('W=$w round $round', round(d['value']/1e6,1), 'M', round(d['ms_per_step'],3), 'ms', d['correct_vs_labels'], 'ahalf', round(r['kernel_ms'],3), r.get('launches_per_step'), 'tables', round(r['pipeline_ms']['comb_tables_aux_stream'],3))" | tee -a $OUT/ab.txt
  done
done
