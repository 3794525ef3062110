mkdir -p gpurun_out/prof_ec3
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ecdsa.py tests/test_gpu_tx_verify.py > gpurun_out/ec_tests.log 2>&1 || { tail -30 gpurun_out/ec_tests.log; exit 1; }
tail -2 gpurun_out/ec_tests.log
timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-txid --no-notary --sigs 100000 > gpurun_out/ec_bench.log 2>&1 || exit 1
grep -o '"ecdsa_mixed[^,]*' gpurun_out/ec_bench.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ec3 -o ec -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-txid --no-notary --sigs 100000 > gpurun_out/prof_ec3/b.log 2>&1
