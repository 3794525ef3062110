#!/bin/bash
# round 5: the host chunk pipeline's Ed25519 tail (finish, bitmap) on a stream of its own with two workspace sets:
# host-entry / group / tx GPU tests, then same-box A/B of the pinned / pageable cfg2 host leg vs the previous commit
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/${1:-r05r}; mkdir -p $OUT
cd $REPO
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_host_entry.py tests/test_gpu_group.py tests/test_gpu_tx_verify.py tests/test_gpu_ecdsa.py > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for round in 1 2; do
  for v in head -; do
    lib=""; [ "$v" != "-" ] && lib="$REPO/build_ab/$v/libcordahip.so"
    CORDAHIP_LIB=$lib timeout -k 10 300 python3 tools/host_sweep.py 1000000 3,4 > $OUT/host_${v}_$round.jsonl 2> $OUT/host.err || { echo "host sweep $v failed"; tail -5 $OUT/host.err; exit 1; }
    sed "s/^/lib=$v round=$round /" $OUT/host_${v}_$round.jsonl | tee -a $OUT/ab.txt
  done
done
