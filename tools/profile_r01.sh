#!/bin/bash
# Round-1 profiling recipe (run on the GPU box from the repo root).  Kernel trace + stats for the
# default bench command, then separate PMC passes (one counter group per run, as gfx950 requires).
set -e
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/prof_r01
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_under_trace.json 2> $OUT/trace.err
SMALL="--n 262144 --steps 2 --warmup 1 --no-cpu-baseline --no-txid --no-ecdsa"
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o p -- python3 bench.py $SMALL > /dev/null 2> $OUT/pmc_fetch.err
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o p -- python3 bench.py $SMALL > /dev/null 2> $OUT/pmc_write.err
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY --output-format csv -d $OUT/pmc_sq -o p -- python3 bench.py $SMALL > /dev/null 2> $OUT/pmc_sq.err
echo profile-done
