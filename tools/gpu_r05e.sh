#!/bin/bash
# Round 5: F(4,3) per-phase s_memtime stamps (item top / steps / epilogue)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05e
mkdir -p $O
timeout -k 10 150 tools/bin/w43_bench_stamps 32 5 > $O/w43_stamps.log 2>&1; rc=$?
[ $rc -le 1 ] || exit $rc
grep -h "stamps\|total" $O/w43_stamps.log
