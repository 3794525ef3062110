#!/bin/bash
# round 5: the host pipeline's per-chunk finish — signatures per inversion chain (CHIP_FINISH_MIN_LANES 49152 = g 4
# for 292k-signature chunks, 32768 = g 8, 16384 = g 16) on the pinned / pageable cfg2 host leg, 2 rounds
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/${1:-r05s}; mkdir -p $OUT
cd $REPO
for round in 1 2; do
  for v in 16384 32768 49152; do
    CHIP_FINISH_MIN_LANES=$v timeout -k 10 300 python3 tools/host_sweep.py 1000000 3,4 > $OUT/host_${v}_$round.jsonl 2> $OUT/host.err || { echo "host sweep $v failed"; tail -5 $OUT/host.err; exit 1; }
    sed "s/^/min_lanes=$v round=$round /" $OUT/host_${v}_$round.jsonl | tee -a $OUT/ab.txt
  done
done
