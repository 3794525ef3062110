#!/bin/bash
# the judged profile of the current tree: tools/profile.sh (kernel trace + SQ/GRBM, FETCH, WRITE, TCC passes)
set -uo pipefail
TAG=${1:-r04}
timeout -k 10 1100 bash tools/profile.sh $TAG || { echo "profile failed"; ls gpurun_out/prof_$TAG; tail -5 gpurun_out/prof_$TAG/*.err; exit 1; }
ls gpurun_out/prof_$TAG
