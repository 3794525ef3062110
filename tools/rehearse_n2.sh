#!/bin/bash
# N=2 rehearsal of bench.py on ONE GPU box: two ranks over gloo sharing cuda:0 (reduced sizes); the
# driver's real N>1 runs use RCCL on separate GPUs.
set -uo pipefail
mkdir -p gpurun_out/n2
export CORDA_BENCH_BACKEND=gloo
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --no-ecdsa --no-notary --cold-n 0 --no-cpu-baseline --no-host-path --txid-n 200000 --sigs 200000 > gpurun_out/n2/b.json 2> gpurun_out/n2/b.err
rc=$?
tail -c 1500 gpurun_out/n2/b.err
exit $rc
