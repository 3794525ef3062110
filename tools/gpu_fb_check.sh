#!/bin/bash
# from-bytes verification correctness: the stx GPU tests (incl. offsets beyond 2 / 4 GiB), then
# tools/bench_stx.py --verify at 1M blobs (3.1 GB of blobs, extra region past 4 GiB)
set -uo pipefail
mkdir -p gpurun_out/fbcheck
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_stx_offsets.py tests/test_gpu_stx.py tests/test_gpu_host_entry.py > gpurun_out/fbcheck/tests.log 2>&1 || { tail -30 gpurun_out/fbcheck/tests.log; exit 1; }
tail -1 gpurun_out/fbcheck/tests.log
timeout -k 10 200 python3 tools/bench_stx.py --n 1000000 --steps 5 --verify > gpurun_out/fbcheck/b.json 2>>gpurun_out/fbcheck/err.log || { tail -5 gpurun_out/fbcheck/err.log; exit 1; }
cat gpurun_out/fbcheck/b.json
