#!/bin/bash
# round 5: host entries with the key pool's exact schemes (no launches for absent schemes) + staging ring opt-in:
# host-entry / group / tx tests; A/B of two register caps (Kryo fused pass 1 at 4 waves, ECDSA q<0> at 3 waves);
# the pinned / pageable host-buffer cfg2 leg
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/${1:-r05j}; mkdir -p $OUT
cd $REPO
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_host_entry.py tests/test_gpu_group.py tests/test_gpu_tx_verify.py tests/test_gpu_cpp_mirror.py tests/test_gpu_ecdsa.py > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for round in 1 2; do
  for v in p1w4 -; do
    lib=""; [ "$v" != "-" ] && lib="$REPO/build_ab/$v/libcordahip.so"
    CORDAHIP_LIB=$lib CHIP_KRYO_FUSED=1 timeout -k 10 200 python3 tools/bench_stx.py --steps 5 >> $OUT/stx.jsonl 2>> $OUT/stx.err || { echo "stx bench $v failed"; tail -5 $OUT/stx.err; exit 1; }
    tail -1 $OUT/stx.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('kryo lib=$v round $round parse', round(d['parse_host_ms'],3), 'ms kernel', round(d['parse_kernel_ms'],3), 'ok', d['status_ok'])" | tee -a $OUT/ab.txt
  done
  for v in q0w3 -; do
    lib=""; [ "$v" != "-" ] && lib="$REPO/build_ab/$v/libcordahip.so"
    CORDAHIP_LIB=$lib timeout -k 10 200 python3 tools/bench_ecdsa.py --steps 10 >> $OUT/ec.jsonl 2>> $OUT/ec.err || { echo "ec bench $v failed"; tail -5 $OUT/ec.err; exit 1; }
    tail -1 $OUT/ec.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ecdsa lib=$v round $round', round(d['sigs_per_s']/1e6,2), 'M', round(d['ms_per_step'],3), 'ms', d['correct'], 'q', round(d['r1_ms'],3), round(d['k1_ms'],3))" | tee -a $OUT/ab.txt
  done
done
timeout -k 10 300 python3 tools/host_sweep.py 1000000 2,3,4,6 > $OUT/host_sweep.jsonl 2> $OUT/host_sweep.err || { echo "host sweep failed"; tail -5 $OUT/host_sweep.err; exit 1; }
cat $OUT/host_sweep.jsonl
