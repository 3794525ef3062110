set -uo pipefail
OUT=gpurun_out/r04b; mkdir -p $OUT
timeout -k 10 120 ./tools/microbench_valu new > $OUT/microbench_valu_new.txt 2>&1 || { echo mb failed; cat $OUT/microbench_valu_new.txt; exit 1; }
cat $OUT/microbench_valu_new.txt
timeout -k 10 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_gpu_ftx.py tests/test_gpu_uniq.py tests/test_gpu_host_entry.py > $OUT/t.log 2>&1 || { echo tests failed; tail -40 $OUT/t.log; exit 1; }
tail -3 $OUT/t.log
