#!/bin/bash
# ahalf restructure: microbench (cndmask forms), Ed25519 GPU parity, same-box A/B of cfg2 (base vs in-tree)
set -uo pipefail
OUT=gpurun_out/${1:-r04c}; mkdir -p $OUT
timeout -k 10 120 ./tools/microbench_valu newest > $OUT/mb.txt 2>&1 || { echo mb failed; cat $OUT/mb.txt; exit 1; }
cat $OUT/mb.txt
timeout -k 10 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_gpu_ed25519.py tests/test_gpu_host_entry.py tests/test_gpu_cfg1_cash.py > $OUT/t.log 2>&1 || { echo tests failed; tail -40 $OUT/t.log; exit 1; }
tail -2 $OUT/t.log
TAG=${1:-r04c} STEPS=10 timeout -k 10 500 bash tools/ab_lib.sh build_ab/base/libcordahip.so - build_ab/base/libcordahip.so - || exit 1
