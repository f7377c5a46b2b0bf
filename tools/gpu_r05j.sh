#!/bin/bash
# Round 5: coalesced STORE epilogue (finisher = output row, quad lanes write one tile row's 64 B)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05j
mkdir -p $O
for r in 1 2; do
  timeout -k 10 200 tools/bin/w43_bench 32 10 > $O/w43_$r.log 2>&1; rc=$?
  [ $rc -le 1 ] || exit $rc
  grep -h "^b\|^e\|total" $O/w43_$r.log | cut -c1-250
done
