#!/bin/bash
# chip_verify_batch (host buffers) in 4 chunks under a kernel + memory-copy trace; timeline of the last call
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/${1:-hostprof}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $OUT/kt -o kt --output-format csv -- \
    python3 $REPO/tools/host_sweep.py 1000000 ${2:-4} > $OUT/sweep.json 2> $OUT/sweep.err || { tail -20 $OUT/sweep.err; exit 1; }
cat $OUT/sweep.json
python3 $REPO/tools/kt_timeline.py $OUT/kt --marker k_chunk_init --occurrence -${2:-4} --count 120 > $OUT/timeline.txt || true
