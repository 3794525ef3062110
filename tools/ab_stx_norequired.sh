set -uo pipefail
cd $GRAFT_REPO_ROOT
for v in - build_ab/nostores/libcordahip.so; do
  lib=""; [ "$v" != "-" ] && lib="$GRAFT_REPO_ROOT/$v"
  CORDAHIP_LIB=$lib timeout -k 10 200 python3 tools/bench_stx.py --steps 5 --no-required > gpurun_out/ns.json 2>>gpurun_out/ns.err || exit 1
  echo "$v $(cat gpurun_out/ns.json)"
done
