#!/bin/bash
# all GPU tests (in-tree: comb radix 2^6), same-box A/B (W=5 cached, W=6 cached = in-tree, affine W=5 / W=6),
# the affine builds' Ed25519 tests, and the full default bench
set -uo pipefail
OUT=gpurun_out/${1:-r04h}; mkdir -p $OUT
timeout -k 10 800 python -u -m pytest -x -v --durations=10 --timeout 150 --timeout-method thread -m gpu tests > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
export TAG=${1:-r04h} STEPS=10
timeout -k 10 900 bash tools/ab_lib.sh build_ab/w5/libcordahip.so - build_ab/a5/libcordahip.so build_ab/a6/libcordahip.so build_ab/w5/libcordahip.so - build_ab/a5/libcordahip.so build_ab/a6/libcordahip.so || exit 1
for v in a5 a6; do
  CORDAHIP_LIB=$PWD/build_ab/$v/libcordahip.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ed25519.py tests/test_gpu_host_entry.py > $OUT/t_$v.log 2>&1; echo "$v: $(tail -1 $OUT/t_$v.log)"
done
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/bench.json')); s=d.get('secondary',d)
print('value', d['value']/1e6, 'ms', d['ms_per_step'], d['correct_vs_labels'])
for k in sorted(s):
    if any(x in k for x in ('per_s','_ms','correct')) and not isinstance(s[k], dict): print(k, s[k])
"
