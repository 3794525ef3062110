#!/bin/bash
# round 5: cfg3 (bench_ecdsa, EC schemes hint): step timeline + PMC passes (issue / wait counters, L2 hits, fetch)
# to see why k_ecdsa_comb_q<0> issues slower than q<1>
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$REPO/gpurun_out/${1:-r05i}; mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_ec -o kt --output-format csv -- python3 $REPO/tools/bench_ecdsa.py --steps 3 > $OUT/ec.json 2> $OUT/ec.err || { echo "ec trace failed"; tail -5 $OUT/ec.err; exit 1; }
python3 $REPO/tools/kt_timeline.py $OUT/kt_ec --marker k_batch_init --count 40 > $OUT/ec_timeline.txt || true
CTRS="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $CTRS -d $OUT/p_sq -o p --output-format csv -- python3 $REPO/tools/bench_ecdsa.py --steps 3 > $OUT/p_sq.json 2> $OUT/p_sq.err || { echo "sq pass failed"; tail -5 $OUT/p_sq.err; exit 1; }
python3 $REPO/tools/pmc_summary.py $(find $OUT/p_sq -name "*counter_collection.csv" | head -1) $OUT/pmc_sq.csv
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/p_tcc -o p --output-format csv -- python3 $REPO/tools/bench_ecdsa.py --steps 3 > $OUT/p_tcc.json 2> $OUT/p_tcc.err || { echo "tcc pass failed"; tail -5 $OUT/p_tcc.err; exit 1; }
python3 $REPO/tools/pmc_summary.py $(find $OUT/p_tcc -name "*counter_collection.csv" | head -1) $OUT/pmc_tcc.csv
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/p_fetch -o p --output-format csv -- python3 $REPO/tools/bench_ecdsa.py --steps 3 > $OUT/p_fetch.json 2> $OUT/p_fetch.err || { echo "fetch pass failed"; tail -5 $OUT/p_fetch.err; exit 1; }
python3 $REPO/tools/pmc_summary.py $(find $OUT/p_fetch -name "*counter_collection.csv" | head -1) $OUT/pmc_fetch.csv
grep -E "comb_q|comb_g|comb_pre|comb_inv|comb_fill|chain" $OUT/pmc_sq.csv $OUT/pmc_tcc.csv $OUT/pmc_fetch.csv
