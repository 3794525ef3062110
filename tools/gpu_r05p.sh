#!/bin/bash
# round 5: ECDSA per-key table fill at 3 waves per SIMD (EC_FILL_WAVES=3) — same-box A/B on cfg3, 3 rounds
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/${1:-r05p}; mkdir -p $OUT
cd $REPO
for round in 1 2 3; do
  for v in fw3 -; do
    lib=""; [ "$v" != "-" ] && lib="$REPO/build_ab/$v/libcordahip.so"
    CORDAHIP_LIB=$lib timeout -k 10 200 python3 tools/bench_ecdsa.py --steps 10 >> $OUT/ec.jsonl 2>> $OUT/ec.err || { echo "ec bench $v failed"; tail -5 $OUT/ec.err; exit 1; }
    tail -1 $OUT/ec.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ecdsa lib=$v round $round', round(d['sigs_per_s']/1e6,2), 'M', round(d['ms_per_step'],3), 'ms', d['correct'], 'q', round(d['r1_ms'],3), round(d['k1_ms'],3), 'front', round(d['front_ms'],3), 'tables', round(d['tables_ms'],3))" | tee -a $OUT/ab.txt
  done
done
