#!/bin/bash
# round 5: Kryo fused walk + ECDSA lane-pair chain: GPU tests, then same-box A/Bs (fused walk, pair chain, per-kernel
# timing events), then the driver's default bench with / without the pinned staging ring
set -uo pipefail
OUT=gpurun_out/${1:-r05f}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_stx.py tests/test_gpu_stx_offsets.py tests/test_gpu_required.py tests/test_gpu_cfg1_cash.py tests/test_gpu_ecdsa.py tests/test_gpu_ref_x509.py tests/test_gpu_key_cache.py tests/test_gpu_ed25519.py > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for round in 1 2; do
  for v in 1 0; do
    CHIP_KRYO_FUSED=$v timeout -k 10 200 python3 tools/bench_stx.py --steps 5 >> $OUT/stx.jsonl 2>> $OUT/stx.err || { echo "stx bench $v failed"; tail -5 $OUT/stx.err; exit 1; }
    tail -1 $OUT/stx.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('fused=$v round $round parse', round(d['parse_host_ms'],3), 'ms kernel', round(d['parse_kernel_ms'],3), 'ok', d['status_ok'], d['nsig'], d['nreq'])" | tee -a $OUT/ab.txt
  done
done
for round in 1 2; do
  for v in 1 0; do
    CHIP_EC_CHAIN_PAIR=$v timeout -k 10 200 python3 tools/bench_ecdsa.py --steps 10 >> $OUT/ab.jsonl 2>> $OUT/ab.err || { echo "bench $v failed"; tail -5 $OUT/ab.err; exit 1; }
    tail -1 $OUT/ab.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('pair=$v round $round', round(d['sigs_per_s']/1e6,2), 'M', round(d['ms_per_step'],3), 'ms', d['correct'], 'tables', round(d['tables_ms'],3), 'front', round(d['front_ms'],3), 'q', round(d['r1_ms']+d['k1_ms'],3))" | tee -a $OUT/ab.txt
  done
done
for round in 1 2; do
  for v in 1 0; do
    CHIP_KERNEL_TIMING=$v timeout -k 10 200 python3 tools/bench_ecdsa.py --ed25519 --n 1000000 --steps 20 --warmup 3 >> $OUT/kt.jsonl 2>> $OUT/kt.err || { echo "kt bench $v failed"; tail -5 $OUT/kt.err; exit 1; }
    tail -1 $OUT/kt.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ktiming=$v round $round', round(d['sigs_per_s']/1e6,2), 'M', round(d['ms_per_step'],3), 'ms', d['correct'])" | tee -a $OUT/ab.txt
  done
done
CHIP_ED_STRAUS_OCC=3 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ed25519.py > $OUT/tests_occ3.log 2>&1 || { echo "occ3 tests failed"; tail -30 $OUT/tests_occ3.log; exit 1; }
tail -1 $OUT/tests_occ3.log
for round in 1 2; do
  for v in 3 1; do
    CHIP_ED_STRAUS_OCC=$v timeout -k 10 300 python3 bench.py --steps 5 --no-txid --no-ecdsa --no-notary --no-cpu-baseline --no-key-cache --no-host-path --no-full-oracle > $OUT/cold_${v}_${round}.json 2> $OUT/cold.err || { echo "cold bench $v failed"; tail -5 $OUT/cold.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$OUT/cold_${v}_${round}.json')); s=d['secondary']
print('straus_occ=$v round $round cold', round(s['ed25519_cold_sigs_per_s']/1e6,2), 'M', round(s['ed25519_cold_ms_per_batch'],3), 'ms straus', round(s['ed25519_cold_straus_ms'],3), 'keyprep', round(s['ed25519_cold_keyprep_ms'],3), s['ed25519_cold_correct'])" | tee -a $OUT/ab.txt
  done
done
cat /sys/fs/cgroup/cpu.max > $OUT/cpu_max.txt 2>&1 || true
for v in 0 1; do
  CHIP_STAGING_RING=$v timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/full_ring$v.json 2> $OUT/full_ring$v.err || { echo "full bench ring=$v failed"; tail -5 $OUT/full_ring$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/full_ring$v.json')); s=d['secondary']
print('full ring=$v', round(d['value']/1e6,1), 'M; pageable', round(s['cfg2_host_path_sigs_per_s']/1e6,1), s['cfg2_host_path_iter_ms'], s['cfg2_host_path_cgroup'], '; pinned', round(s['cfg2_host_path_pinned_sigs_per_s']/1e6,1), s['cfg2_host_path_pinned_iter_ms'])" | tee -a $OUT/ab.txt
done
