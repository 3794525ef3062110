set -uo pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ec4
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ec_field.py tests/test_gpu_ecdsa.py tests/test_gpu_ref_x509.py > gpurun_out/ec4/tests.log 2>&1 || { tail -30 gpurun_out/ec4/tests.log; exit 1; }
tail -2 gpurun_out/ec4/tests.log
bash tools/ab_ecdsa.sh ab4
