set -euo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/kt_r02a
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 $REPO/bench.py --steps 3 --warmup 1 --no-txid --no-notary --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
