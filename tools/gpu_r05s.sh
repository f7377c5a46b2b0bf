#!/bin/bash
# Round 5: POOL2 epilogue store pattern ablation (abl32: coalesced)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05s
mkdir -p $O
for r in 1 2; do
  for v in "" _abl32; do
    timeout -k 10 200 tools/bin/w43_bench$v 32 10 > $O/w43${v}_$r.log 2>&1; rc=$?
    [ $rc -le 1 ] || exit $rc
    echo "== w43$v run $r: $(grep -h '^b.c2' $O/w43${v}_$r.log | awk '{printf "%s %s  ", $1, $11}')"
  done
done
