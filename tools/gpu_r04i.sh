#!/bin/bash
# key cache: its GPU tests first, then all GPU tests and the full default bench
set -uo pipefail
OUT=gpurun_out/${1:-r04i}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_gpu_key_cache.py > $OUT/kc_tests.log 2>&1 || { echo "key cache tests failed"; tail -30 $OUT/kc_tests.log; exit 1; }
tail -1 $OUT/kc_tests.log
timeout -k 10 800 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 700 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/bench.json')); s=d.get('secondary',d)
print('value', d['value']/1e6, 'ms', d['ms_per_step'], d['correct_vs_labels'])
for k in sorted(s):
    if any(x in k for x in ('per_s','_ms','correct', 'pipeline')): print(k, s[k])
"
