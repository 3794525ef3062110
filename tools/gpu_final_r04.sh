#!/bin/bash
# round-4 final tree: every GPU test, smoke(), the default bench line
set -uo pipefail
OUT=gpurun_out/${1:-final_r04}; mkdir -p $OUT
timeout -k 10 800 python -u -m pytest -x -v --durations=15 --timeout 200 --timeout-method thread -m gpu tests > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 700 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/bench.json')); s=d['secondary']; print('value', d['value']/1e6, 'ms', d['ms_per_step'], d['correct_vs_labels'], 'bytes', s['cfg4_from_bytes_correct'], s['cfg4_from_bytes_verified_tx_per_s']/1e6, s['stx_parse_ms'], s['stx_parse_roofline'].get('traffic'))"
