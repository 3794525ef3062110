set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/stx_pmc_b
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_IFETCH SQ_ACTIVE_INST_ANY SQ_INSTS_VALU -d $OUT/w -o w --output-format csv -- python3 $REPO/tools/bench_stx.py --steps 1 > $OUT/b.json 2> $OUT/b.err || { tail -5 $OUT/b.err; exit 1; }
python3 $REPO/tools/pmc_summary.py $(find $OUT/w -name "*counter_collection.csv" | head -1) $OUT/pmc_wait.csv
grep -E "stx" $OUT/pmc_wait.csv
