#!/bin/bash
# round 5: host pipeline copy/check stream at high priority (CHIP_HCS_PRIORITY=1) vs default, cfg2 host legs
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/${1:-r05t}; mkdir -p $OUT
cd $REPO
for round in 1 2; do
  for v in 1 0; do
    CHIP_HCS_PRIORITY=$v timeout -k 10 300 python3 tools/host_sweep.py 1000000 4 > $OUT/host_${v}_$round.jsonl 2> $OUT/host.err || { echo "host sweep $v failed"; tail -5 $OUT/host.err; exit 1; }
    sed "s/^/hcs_prio=$v round=$round /" $OUT/host_${v}_$round.jsonl | tee -a $OUT/ab.txt
  done
done
