set -uo pipefail
mkdir -p gpurun_out/hostcmp
A="--steps 3 --warmup 1 --cold-n 0 --no-txid --no-ecdsa --no-notary --no-cpu-baseline"
CHIP_HOST_CHUNKS=1 timeout -k 10 300 python bench.py $A > gpurun_out/hostcmp/c1.json 2> gpurun_out/hostcmp/c1.err && \
timeout -k 10 300 python bench.py $A > gpurun_out/hostcmp/c4.json 2> gpurun_out/hostcmp/c4.err && \
for f in c1 c4; do python3 -c "import json; s=json.load(open('gpurun_out/hostcmp/$f.json'))['secondary']; print('$f', s['cfg2_host_path_ms'], s['cfg2_host_path_pinned_ms'])"; done
