#!/bin/bash
# Uniqueness GPU check: uniq tests, then the cfg5 notary leg alone under a kernel trace.
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-uniq}
OUT=$REPO/gpurun_out/$TAG
mkdir -p $OUT
cd $REPO
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_uniq.py tests/test_gpu_uniq_dist.py tests/test_gpu_cpp_mirror.py > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 $REPO/bench.py --sigs 65536 --cold-n 0 --no-txid --no-ecdsa --no-cpu-baseline --no-host-path > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/bench.json')); s=d['secondary']
print({k: s[k] for k in s if k.startswith('notary')})"
