#!/bin/bash
# round 5: the register caps as defaults (ECDSA q<0> 3 waves, Kryo fused pass 1 4 waves): ECDSA / Kryo / key-cache
# GPU tests, then A/B of a k_ecdsa_comb_g cap (3 waves) over the cfg3 shape
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/${1:-r05k}; mkdir -p $OUT
cd $REPO
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ecdsa.py tests/test_gpu_ref_x509.py tests/test_gpu_key_cache.py tests/test_gpu_stx.py tests/test_gpu_stx_offsets.py tests/test_gpu_required.py tests/test_gpu_sig_dist.py > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for round in 1 2; do
  for v in g3 -; do
    lib=""; [ "$v" != "-" ] && lib="$REPO/build_ab/$v/libcordahip.so"
    CORDAHIP_LIB=$lib timeout -k 10 200 python3 tools/bench_ecdsa.py --steps 10 >> $OUT/ec.jsonl 2>> $OUT/ec.err || { echo "ec bench $v failed"; tail -5 $OUT/ec.err; exit 1; }
    tail -1 $OUT/ec.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ecdsa lib=$v round $round', round(d['sigs_per_s']/1e6,2), 'M', round(d['ms_per_step'],3), 'ms', d['correct'], 'q', round(d['r1_ms'],3), round(d['k1_ms'],3), 'front', round(d['front_ms'],3))" | tee -a $OUT/ab.txt
  done
done
