#!/bin/bash
# all GPU tests, then a same-box A/B of cfg2 (base vs in-tree) and the full default bench on the in-tree build
set -uo pipefail
OUT=gpurun_out/${1:-r04f}; mkdir -p $OUT
timeout -k 10 800 python -u -m pytest -x -v --durations=15 --timeout 150 --timeout-method thread -m gpu tests > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
TAG=${1:-r04f} STEPS=10 timeout -k 10 400 bash tools/ab_lib.sh build_ab/base/libcordahip.so - || exit 1
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/bench.json')); s=d.get('secondary',d)
print('value', d['value']/1e6, 'ms', d['ms_per_step'])
for k in sorted(s):
    if any(x in k for x in ('per_s','_ms','correct','GBps')) and not isinstance(s[k], dict): print(k, s[k])
"
