#!/bin/bash
# round 5: cfg2 register caps (k_ed_comb_bhalf at 3 waves, k_ed_comb_finish at 4) — same-box A/B, 3 rounds
set -uo pipefail
REPO=${GRAFT_REPO_ROOT:-$(pwd)}
cd $REPO
for round in 1 2 3; do
  TAG=${1:-r05l} STEPS=10 bash tools/ab_lib.sh build_ab/bh3/libcordahip.so build_ab/fin4/libcordahip.so build_ab/bhfin/libcordahip.so - || exit 1
done
