#!/bin/bash
# rocprofv3 passes for the judged profiles (run on the GPU box through gpurun):
#   1. kernel trace + stats over the default bench command (every leg, full sizes)
#   2-5. PMC passes, one counter group per run (kernel trace only, no other trace domains), over
#        every leg at full size but fewer steps: SQ issue counters + GRBM clock, FETCH_SIZE, WRITE_SIZE, L2 hits
# Outputs under gpurun_out/prof_<tag>/ with the condensed CSVs bench.py reads (pmc_sq.csv, issue_model.csv,
# pmc_fetch_size.csv, pmc_write_size.csv, pmc_tcc.csv, kernel_stats.csv); copy those into profiles/<round>/.
set -euo pipefail
TAG=${1:-run}
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
BENCH_PMC="$REPO/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-path --no-notary-check"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- \
    python3 "$REPO/bench.py" --steps 5 --warmup 2 > "$OUT/bench_kt.json" 2> "$OUT/bench_kt.err"
cp "$(find "$OUT/kt" -name "kt_kernel_stats.csv" | head -1)" "$OUT/kernel_stats.csv"
echo "kernel trace done"
pass() {   # pass <name> <counters...>
    local name=$1; shift
    timeout -s KILL 400 rocprofv3 --kernel-trace --pmc "$@" -d "$OUT/$name" -o "$name" --output-format csv -- \
        python3 $BENCH_PMC > "$OUT/bench_$name.json" 2> "$OUT/bench_$name.err"
    find "$OUT/$name" -name "*counter_collection.csv" | head -1
}
# 7 SQ + 2 GRBM counters (limits: 8 SQ, 2 GRBM per pass)
f=$(pass sq SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY \
    GRBM_GUI_ACTIVE GRBM_COUNT)
python3 "$REPO/tools/pmc_summary.py" "$f" "$OUT/pmc_sq.csv"
python3 "$REPO/tools/issue_summary.py" "$f" "$OUT/issue_model.csv"
echo "sq pass done"
f=$(pass fetch FETCH_SIZE); python3 "$REPO/tools/pmc_summary.py" "$f" "$OUT/pmc_fetch_size.csv"
echo "fetch pass done"
f=$(pass write WRITE_SIZE); python3 "$REPO/tools/pmc_summary.py" "$f" "$OUT/pmc_write_size.csv"
echo "write pass done"
f=$(pass tcc TCC_HIT_sum TCC_MISS_sum); python3 "$REPO/tools/pmc_summary.py" "$f" "$OUT/pmc_tcc.csv"
echo "tcc pass done"
