#!/bin/bash
# ECDSA-focused GPU check: field arithmetic harness, ECDSA parity tests, then a cfg3 kernel trace.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-ec}
OUT=$REPO/gpurun_out/$TAG
mkdir -p $OUT
cd $REPO
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ec_field.py \
    tests/test_gpu_ecdsa.py tests/test_gpu_ref_x509.py > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 $REPO/bench.py --steps 3 --warmup 1 --no-txid --no-notary --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json | head -c 1500
