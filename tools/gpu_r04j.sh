#!/bin/bash
# early hash/[S]B (in-tree) vs HEAD (build_ab/head) vs in-tree with CHIP_ED_NO_EARLY=1; Ed25519 GPU tests first
set -uo pipefail
OUT=gpurun_out/${1:-r04j}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_gpu_ed25519.py tests/test_gpu_host_entry.py tests/test_gpu_key_cache.py tests/test_gpu_stx.py > $OUT/t.log 2>&1 || { echo "tests failed"; tail -30 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
export TAG=${1:-r04j} STEPS=10
for r in 1 2; do
  timeout -k 10 300 bash tools/ab_lib.sh - build_ab/head/libcordahip.so build_ab/ah3/libcordahip.so || exit 1
  CHIP_ED_NO_EARLY=1 timeout -k 10 300 bash tools/ab_lib.sh - || exit 1
done
