#!/bin/bash
# same-box A/B of comb variants: in-tree (cached rows, W=5) vs affine rows (a5, a6) and cached radix 2^6 / 2^7
# (w6, w7); then the Ed25519 GPU tests on the affine build
set -uo pipefail
export TAG=${1:-abw}
export STEPS=10
timeout -k 10 900 bash tools/ab_lib.sh - build_ab/a5/libcordahip.so build_ab/a6/libcordahip.so build_ab/w6/libcordahip.so build_ab/w7/libcordahip.so - build_ab/a5/libcordahip.so build_ab/a6/libcordahip.so build_ab/w6/libcordahip.so || exit 1
CORDAHIP_LIB=$PWD/build_ab/a5/libcordahip.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ed25519.py tests/test_gpu_host_entry.py > gpurun_out/$TAG/t_a5.log 2>&1; tail -2 gpurun_out/$TAG/t_a5.log
CORDAHIP_LIB=$PWD/build_ab/a6/libcordahip.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ed25519.py tests/test_gpu_host_entry.py > gpurun_out/$TAG/t_a6.log 2>&1; tail -2 gpurun_out/$TAG/t_a6.log
