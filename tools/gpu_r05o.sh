#!/bin/bash
# round 5: ECDSA front end — signature staged in LDS (independent loads, no dependent byte chain), DER integers by
# destination byte, SHA-256 blocks fetched one ahead with dwordx4 loads: ECDSA GPU tests, then A/B vs the previous
# commit (build_ab/head) on the cfg3 shape; Kryo post / required caps (pr5, p5) if time allows
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/${1:-r05o}; mkdir -p $OUT
cd $REPO
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ecdsa.py tests/test_gpu_ref_x509.py tests/test_gpu_key_cache.py tests/test_gpu_host_entry.py tests/test_gpu_tx_verify.py > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for round in 1 2 3; do
  for v in head -; do
    lib=""; [ "$v" != "-" ] && lib="$REPO/build_ab/$v/libcordahip.so"
    CORDAHIP_LIB=$lib timeout -k 10 200 python3 tools/bench_ecdsa.py --steps 10 >> $OUT/ec.jsonl 2>> $OUT/ec.err || { echo "ec bench $v failed"; tail -5 $OUT/ec.err; exit 1; }
    tail -1 $OUT/ec.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ecdsa lib=$v round $round', round(d['sigs_per_s']/1e6,2), 'M', round(d['ms_per_step'],3), 'ms', d['correct'], 'q', round(d['r1_ms'],3), round(d['k1_ms'],3), 'front', round(d['front_ms'],3))" | tee -a $OUT/ab.txt
  done
done
for round in 1 2; do
  for v in pr5 p5 -; do
    lib=""; [ "$v" != "-" ] && lib="$REPO/build_ab/$v/libcordahip.so"
    CORDAHIP_LIB=$lib timeout -k 10 200 python3 tools/bench_stx.py --steps 5 >> $OUT/stx.jsonl 2>> $OUT/stx.err || { echo "stx bench $v failed"; tail -5 $OUT/stx.err; exit 1; }
    tail -1 $OUT/stx.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('kryo lib=$v round $round parse', round(d['parse_host_ms'],3), 'ms kernel', round(d['parse_kernel_ms'],3), 'ok', d['status_ok'])" | tee -a $OUT/ab.txt
  done
done
