#!/bin/bash
# reordered early pipeline + priorities + one init kernel: GPU tests, same-box A/B vs HEAD, then the step timeline
set -uo pipefail
OUT=gpurun_out/${1:-r04m}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_gpu_ed25519.py tests/test_gpu_ecdsa.py tests/test_gpu_host_entry.py tests/test_gpu_key_cache.py tests/test_gpu_stx.py tests/test_gpu_sig_dist.py > $OUT/t.log 2>&1 || { echo "tests failed"; tail -30 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
export TAG=${1:-r04m} STEPS=10
for r in 1 2 3; do
  timeout -k 10 300 bash tools/ab_lib.sh - build_ab/nopair/libcordahip.so || exit 1
done
timeout -k 10 400 bash tools/gpu_tl.sh ${1:-r04m}_tl | tail -30
