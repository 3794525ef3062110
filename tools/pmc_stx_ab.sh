#!/bin/bash
# WRITE_SIZE / FETCH_SIZE of the Kryo parse kernels (tools/bench_stx.py, 2 steps) for the in-tree library and a
# variant ($1): which part of pass 2's writes are the index stores (KRYO_NO_STORES variant)
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/${TAG:-pmcstx}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for v in - "$1"; do
  lib=""; [ "$v" != "-" ] && lib="$REPO/$v"
  tag=$([ "$v" = "-" ] && echo base || echo variant)
  for c in WRITE_SIZE FETCH_SIZE; do
    CORDAHIP_LIB=$lib timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $c -d $OUT/${tag}_$c -o x --output-format csv -- python3 $REPO/tools/bench_stx.py --steps 2 > $OUT/${tag}_$c.json 2> $OUT/${tag}_$c.err || { tail -5 $OUT/${tag}_$c.err; exit 1; }
    python3 $REPO/tools/pmc_summary.py $(find $OUT/${tag}_$c -name "*counter_collection.csv" | head -1) $OUT/${tag}_$c.csv
    grep "stx_parse" $OUT/${tag}_$c.csv | sed "s/^/$tag /"
  done
done
