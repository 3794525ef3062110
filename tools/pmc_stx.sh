#!/bin/bash
# PMC passes over tools/bench_stx.py (one counter group per run, kernel trace only): SQ instruction mix,
# FETCH_SIZE, WRITE_SIZE of the Kryo front-end kernels.  Summaries -> gpurun_out/<tag>/pmc_*.csv
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/${1:-stx_pmc}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
pass() {
    local name=$1; shift
    timeout -s KILL 240 rocprofv3 --kernel-trace --pmc "$@" -d $OUT/$name -o $name --output-format csv -- \
        python3 $REPO/tools/bench_stx.py --steps 1 > $OUT/bench_$name.json 2> $OUT/bench_$name.err || { tail -5 $OUT/bench_$name.err; return 1; }
    python3 $REPO/tools/pmc_summary.py $(find $OUT/$name -name "*counter_collection.csv" | head -1) $OUT/pmc_$name.csv
}
pass sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES && \
pass fetch FETCH_SIZE && pass write WRITE_SIZE
for f in $OUT/pmc_*.csv; do grep -E "stx|key_check" $f; done
