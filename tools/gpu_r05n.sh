#!/bin/bash
# round 5: Kryo A/B — k_stx_post / k_stx_required register caps (5 waves), and the post-in-pass-1 level (FUSED=2)
# now that pass 1 is capped at 4 waves
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/${1:-r05n}; mkdir -p $OUT
cd $REPO
for round in 1 2; do
  for v in pr5 p5 - fused2; do
    lib=""; F=1
    case $v in pr5|p5) lib="$REPO/build_ab/$v/libcordahip.so";; fused2) F=2;; esac
    CORDAHIP_LIB=$lib CHIP_KRYO_FUSED=$F timeout -k 10 200 python3 tools/bench_stx.py --steps 5 --verify >> $OUT/stx.jsonl 2>> $OUT/stx.err || { echo "stx bench $v failed"; tail -5 $OUT/stx.err; exit 1; }
    tail -1 $OUT/stx.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('kryo $v round $round parse', round(d['parse_host_ms'],3), 'ms kernel', round(d['parse_kernel_ms'],3), 'ok', d['status_ok'], d.get('verify_correct'))" | tee -a $OUT/ab.txt
  done
done
