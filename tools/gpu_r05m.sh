#!/bin/bash
# round 5: Kryo transposes with a guessed owner search, k_stx_dechunk with 16 lanes per transaction: stx GPU tests
# (incl. > 4 GiB offsets), A/B dechunk width 16 / 64, then the front end's timeline
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/${1:-r05m}; mkdir -p $OUT
cd $REPO
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_stx.py tests/test_gpu_stx_offsets.py tests/test_gpu_required.py tests/test_gpu_cfg1_cash.py > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for round in 1 2; do
  for v in 16 64; do
    CHIP_KRYO_DECHUNK_W=$v timeout -k 10 200 python3 tools/bench_stx.py --steps 5 --verify >> $OUT/stx.jsonl 2>> $OUT/stx.err || { echo "stx bench $v failed"; tail -5 $OUT/stx.err; exit 1; }
    tail -1 $OUT/stx.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('dechunk_w=$v round $round parse', round(d['parse_host_ms'],3), 'ms kernel', round(d['parse_kernel_ms'],3), 'ok', d['status_ok'], d.get('verify_correct'))" | tee -a $OUT/ab.txt
  done
done
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_stx -o kt --output-format csv -- python3 $REPO/tools/bench_stx.py --steps 3 > $OUT/stx_kt.json 2> $OUT/stx_kt.err || { echo "stx trace failed"; tail -5 $OUT/stx_kt.err; exit 1; }
python3 $REPO/tools/kt_timeline.py $OUT/kt_stx --count 70 > $OUT/stx_timeline.txt || true
head -25 $OUT/stx_timeline.txt
