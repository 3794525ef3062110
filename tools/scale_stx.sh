#!/bin/bash
# pass-1 / pass-2 kernel times of the Kryo front end at several batch sizes (is the walk throughput- or
# latency-bound?), from kernel traces of tools/bench_stx.py --no-required
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp
for n in 125000 250000 500000 1000000; do
  OUT=$REPO/gpurun_out/scale_stx/$n
  mkdir -p $OUT
  timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/kt -o kt --output-format csv -- python3 $REPO/tools/bench_stx.py --n $n --steps 3 --no-required > $OUT/b.json 2> $OUT/b.err || exit 1
  echo "n=$n $(python3 $REPO/tools/kt_timeline.py $OUT/kt --count 40 | grep -E 'k_stx_parse|key_insert' | awk '{print $2, $NF}' | tr '\n' ' ')"
done
