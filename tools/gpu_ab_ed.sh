#!/bin/bash
# Ed25519 kernel change: GPU parity (Ed25519 / host entry / cash tests), then a same-box A/B of cfg2
# (build_ab/base vs the in-tree library, twice each).  tools/gpu_ab_ed.sh <tag>
set -uo pipefail
OUT=gpurun_out/${1:-ab_ed}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_gpu_ed25519.py tests/test_gpu_host_entry.py tests/test_gpu_cfg1_cash.py tests/test_gpu_tx_verify.py > $OUT/t.log 2>&1 || { echo tests failed; tail -40 $OUT/t.log; exit 1; }
tail -2 $OUT/t.log
TAG=${1:-ab_ed} STEPS=10 timeout -k 10 500 bash tools/ab_lib.sh build_ab/base/libcordahip.so - build_ab/base/libcordahip.so - || exit 1
