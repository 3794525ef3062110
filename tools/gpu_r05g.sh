#!/bin/bash
# round 5: Kryo front-end timeline (fused walk), cfg3 step timeline (why q<0> issues slower), staging-ring copy threads
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/${1:-r05g}; mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_stx -o kt --output-format csv -- python3 $REPO/tools/bench_stx.py --steps 3 > $OUT/stx.json 2> $OUT/stx.err || { echo "stx trace failed"; tail -5 $OUT/stx.err; exit 1; }
python3 $REPO/tools/kt_timeline.py $OUT/kt_stx --count 70 > $OUT/stx_timeline.txt || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_ec -o kt --output-format csv -- python3 $REPO/tools/bench_ecdsa.py --steps 3 > $OUT/ec.json 2> $OUT/ec.err || { echo "ec trace failed"; tail -5 $OUT/ec.err; exit 1; }
python3 $REPO/tools/kt_timeline.py $OUT/kt_ec --marker k_batch_init --count 40 > $OUT/ec_timeline.txt || true
cd $REPO
for round in 1 2; do
  for v in 16 8 0; do
    if [ $v = 0 ]; then R=0; T=8; else R=1; T=$v; fi
    CHIP_STAGING_RING=$R CHIP_COPY_THREADS=$T timeout -k 10 300 python3 bench.py --steps 3 --no-txid --no-ecdsa --no-notary --cold-n 0 --no-cpu-baseline --no-key-cache --no-full-oracle > $OUT/host_${v}_${round}.json 2> $OUT/host.err || { echo "host bench $v failed"; tail -5 $OUT/host.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$OUT/host_${v}_${round}.json')); s=d['secondary']
print('ring=$R threads=$T round $round pageable', round(s['cfg2_host_path_sigs_per_s']/1e6,1), s['cfg2_host_path_iter_ms'], '; pinned', round(s['cfg2_host_path_pinned_sigs_per_s']/1e6,1), s['cfg2_host_path_pinned_iter_ms'])" | tee -a $OUT/ab.txt
  done
done
