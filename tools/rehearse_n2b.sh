#!/bin/bash
# N=2 rehearsal of every bench leg on ONE GPU box (two ranks over gloo sharing cuda:0, reduced sizes), including the
# host-buffer legs (median of 5 calls, cgroup probe) and the notary / ECDSA legs
set -uo pipefail
mkdir -p gpurun_out/n2b
export CORDA_BENCH_BACKEND=gloo
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 2 --warmup 1 --cold-n 20000 --no-cpu-baseline --txid-n 100000 --sigs 200000 --ecdsa-n 200000 --notary-tx 200000 --notary-pre 500000 > gpurun_out/n2b/b.json 2> gpurun_out/n2b/b.err
rc=$?
tail -c 1500 gpurun_out/n2b/b.err
python3 -c "
import json; t=open('gpurun_out/n2b/b.json').read().splitlines(); d=json.loads([l for l in t if l.startswith('{')][-1])
print('n_gpus', d['n_gpus'], 'value', round(d['value']/1e6,2), d['correct_vs_labels'], 'host', round(d['secondary'].get('cfg2_host_path_sigs_per_s',0)/1e6,1))" || true
exit $rc
