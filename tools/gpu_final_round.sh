#!/bin/bash
# final tree of a round: every GPU test, smoke(), the default bench line (the driver's command)
set -uo pipefail
OUT=gpurun_out/${1:-final}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --durations=15 --timeout 300 --timeout-method thread -m gpu tests > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 700 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/bench.json')); s=d['secondary']
print('value', round(d['value']/1e6,2), 'ms', round(d['ms_per_step'],3), d['correct_vs_labels'])
for k in ('cfg2_host_path_sigs_per_s','cfg2_host_path_pinned_sigs_per_s','ed25519_cold_sigs_per_s','cfg2_key_cache_sigs_per_s','ecdsa_mixed_sigs_per_s','cfg4_from_bytes_verified_tx_per_s','txids_per_s','notary_commit_ms','notary_rounds'):
    v=s.get(k); print(k, (round(v/1e6,2) if k.endswith('_per_s') else round(v,3)) if isinstance(v,(int,float)) else v)
print('stx_parse_ms', s.get('stx_parse_ms'), 'notary', s.get('notary_commit_ms'))"
