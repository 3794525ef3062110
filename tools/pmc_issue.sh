#!/bin/bash
# Issue-side counters of the cfg2 Ed25519 kernels (and the VALU microbench) — where each kernel's wave-cycles go:
# issuing VALU, waiting at s_waitcnt (memory), or waiting for an issue slot — plus GRBM_GUI_ACTIVE for the
# effective clock (GRBM_GUI_ACTIVE / 8 / wall, MI355X_MICROARCH.md:497).  One pass per library given
# (- = the in-tree build), then one over the microbench.  tools/pmc_issue.sh <tag> [lib...]
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-issue}; shift
OUT=$REPO/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-host-path --no-notary --no-ecdsa --no-txid --cold-n 0"
CTRS="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for v in "${@:--}"; do
  i=$((i+1))
  lib=""; [ "$v" != "-" ] && lib="$REPO/$v"
  export CORDAHIP_LIB=$lib
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $CTRS -d $OUT/p$i -o p$i --output-format csv -- python3 $REPO/bench.py $ARGS > $OUT/b$i.json 2> $OUT/b$i.err || { echo "pass $i failed"; tail -5 $OUT/b$i.err; exit 1; }
  python3 $REPO/tools/pmc_summary.py $(find $OUT/p$i -name "*counter_collection.csv" | head -1) $OUT/pmc_issue_$i.csv
  echo "== $v"; grep -E "k_ed_comb_(ahalf|bhalf|hash)" $OUT/pmc_issue_$i.csv
done
unset CORDAHIP_LIB
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $OUT/mb -o mb --output-format csv -- $REPO/tools/microbench_valu > $OUT/mb_under_pmc.txt 2> $OUT/mb.err || { echo "mb pass failed"; tail -5 $OUT/mb.err; exit 1; }
python3 $REPO/tools/pmc_summary.py $(find $OUT/mb -name "*counter_collection.csv" | head -1) $OUT/pmc_mb.csv
find $OUT -name "*kernel_trace.csv" | head -5
