#!/bin/bash
# Round 5: is the STORE epilogue's scattered 16-byte store pattern what makes it 2x POOL2's? (abl16: coalesced)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05i
mkdir -p $O
for r in 1 2; do
  for v in "" _abl16; do
    timeout -k 10 200 tools/bin/w43_bench$v 32 10 > $O/w43${v}_$r.log 2>&1; rc=$?
    [ $rc -le 1 ] || exit $rc
    echo "== w43$v run $r"; grep -h "^b.c1\|total" $O/w43${v}_$r.log | cut -c1-60
  done
done
