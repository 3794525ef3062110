#!/bin/bash
# round 5: Kryo pass 1 with k_stx_post's work folded in (CHIP_KRYO_FUSED=2): stx GPU tests, A/B 2/1/0,
# then a kernel + memory-copy trace of the pinned host-buffer cfg2 path (chunk overlap)
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/${1:-r05h}; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_stx.py tests/test_gpu_stx_offsets.py tests/test_gpu_required.py tests/test_gpu_cfg1_cash.py tests/test_gpu_group.py > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for round in 1 2; do
  for v in 2 1 0; do
    CHIP_KRYO_FUSED=$v timeout -k 10 200 python3 tools/bench_stx.py --steps 5 --verify >> $OUT/stx.jsonl 2>> $OUT/stx.err || { echo "stx bench $v failed"; tail -5 $OUT/stx.err; exit 1; }
    tail -1 $OUT/stx.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('fused=$v round $round parse', round(d['parse_host_ms'],3), 'ms kernel', round(d['parse_kernel_ms'],3), 'ok', d['status_ok'], d.get('verify_correct'), d['nsig'], d['nreq'])" | tee -a $OUT/ab.txt
  done
done
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $OUT/kt_stx -o kt --output-format csv -- python3 $REPO/tools/bench_stx.py --steps 3 > $OUT/stx_kt.json 2> $OUT/stx_kt.err || { echo "stx trace failed"; tail -5 $OUT/stx_kt.err; exit 1; }
python3 $REPO/tools/kt_timeline.py $OUT/kt_stx --count 70 > $OUT/stx_timeline.txt || true
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $OUT/kt_host -o kt --output-format csv -- python3 $REPO/tools/host_sweep.py 1000000 4 > $OUT/host.json 2> $OUT/host.err || { echo "host trace failed"; tail -5 $OUT/host.err; exit 1; }
python3 $REPO/tools/kt_timeline.py $OUT/kt_host --marker k_chunk_init --occurrence -5 --count 90 > $OUT/host_timeline.txt || true
cat $OUT/host.json
