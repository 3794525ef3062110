set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/lm_a
mkdir -p $OUT
cd $REPO
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_stx.py tests/test_gpu_cfg1_cash.py tests/test_gpu_required.py > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python tools/bench_stx.py --steps 5 > $OUT/bench_stx.json 2> $OUT/bench_stx.err || { tail -5 $OUT/bench_stx.err; exit 1; }
cat $OUT/bench_stx.json
export TMPDIR=/tmp
cd /tmp
for c in WRITE_SIZE FETCH_SIZE; do
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $c -d $OUT/$c -o x --output-format csv -- python3 $REPO/tools/bench_stx.py --steps 2 > $OUT/$c.json 2> $OUT/$c.err || { tail -5 $OUT/$c.err; exit 1; }
  python3 $REPO/tools/pmc_summary.py $(find $OUT/$c -name "*counter_collection.csv" | head -1) $OUT/$c.csv
  grep "stx_parse\|stx_lm" $OUT/$c.csv
done
