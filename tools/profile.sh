#!/bin/bash
# rocprofv3 passes for the judged profiles (run on the GPU box through gpurun):
#   1. kernel trace + stats over the default bench command
#   2-4. PMC passes (one counter group per run, kernel-trace only) over a reduced bench
# Outputs under gpurun_out/prof_<tag>/; copy the summaries into profiles/<round>/.
set -euo pipefail
TAG=${1:-run}
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
BENCH_SMALL="$REPO/bench.py --steps 2 --warmup 1 --no-ecdsa --no-notary --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- \
    python3 "$REPO/bench.py" --steps 5 --warmup 2 > "$OUT/bench_kt.json" 2> "$OUT/bench_kt.err"
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_WAVE_CYCLES \
    SQ_BUSY_CYCLES -d "$OUT/sq" -o sq --output-format csv -- python3 $BENCH_SMALL > "$OUT/bench_sq.json" 2> "$OUT/bench_sq.err"
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/fetch" -o fetch --output-format csv -- \
    python3 $BENCH_SMALL > "$OUT/bench_fetch.json" 2> "$OUT/bench_fetch.err"
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/write" -o write --output-format csv -- \
    python3 $BENCH_SMALL > "$OUT/bench_write.json" 2> "$OUT/bench_write.err"
find "$OUT" -name "*.csv" | head -50
