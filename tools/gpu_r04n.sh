#!/bin/bash
# Round 4 final: profiles of the final tree (headline winograd, config 3,
# config 4: kernel trace + FETCH / WRITE / MFMA passes) and the full bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04n
mkdir -p $OUT
NO_FULL=1 PRECISIONS="winograd" LEGS="config3 config4" timeout -k 10 1000 bash tools/profile_round.sh > $OUT/prof.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > $OUT/bench_full.log 2>&1 || exit $?
tail -c 300 $OUT/bench_full.log
echo ALLDONE
