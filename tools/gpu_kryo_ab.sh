#!/bin/bash
# Kryo front end: stx parity tests on the in-tree build (deferred de-chunk copies), then in-tree vs the
# in-place-copy build (KRYO_DEFER_COPY=0), twice
set -uo pipefail
export TAG=${1:-kryo_ab} STEPS=5
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_stx.py tests/test_gpu_host_entry.py > gpurun_out/$TAG/tests.log 2>&1 || { tail -30 gpurun_out/$TAG/tests.log; exit 1; }
tail -3 gpurun_out/$TAG/tests.log
for r in ${ROUNDS:-1 2}; do
  timeout -k 10 400 bash tools/ab_stx.sh - build_ab/inplace/libcordahip.so || exit 1
done
