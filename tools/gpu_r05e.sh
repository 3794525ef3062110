#!/bin/bash
# round 5: host-entry tests (pinned staging ring), then A/B of the cfg2 host-buffer leg with / without the ring
set -uo pipefail
OUT=gpurun_out/${1:-r05e}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_host_entry.py tests/test_gpu_group.py tests/test_gpu_uniq.py tests/test_gpu_stx.py tests/test_gpu_txid.py > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for round in 1 2; do
  for v in 1 0; do
    CHIP_STAGING_RING=$v timeout -k 10 200 python bench.py --steps 5 --no-txid --no-ecdsa --no-notary --cold-n 0 --no-cpu-baseline --no-key-cache > $OUT/b_${v}_$round.json 2> $OUT/b_${v}_$round.err || { echo "bench $v failed"; tail -5 $OUT/b_${v}_$round.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$OUT/b_${v}_$round.json')); s=d['secondary']
print('ring=$v round $round', 'dev', round(d['value']/1e6,1), 'M; host pageable', round(s['cfg2_host_path_sigs_per_s']/1e6,1), 'M', round(s['cfg2_host_path_ms'],2), 'ms', s['cfg2_host_path_correct'], '; pinned', round(s['cfg2_host_path_pinned_sigs_per_s']/1e6,1), 'M', round(s['cfg2_host_path_pinned_ms'],2), 'ms')" | tee -a $OUT/ab.txt
  done
done
