#!/bin/bash
# Round 5: items per F(4,3) workgroup (SEDX_W43_ITEMS 1 / 2 default / 3 / 4), two alternating rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05n
mkdir -p $O
for r in 1 2; do
  for v in "" _it4 _it6 _it8 _it16; do
    timeout -k 10 200 tools/bin/w43_bench$v 32 10 > $O/w43${v}_$r.log 2>&1; rc=$?
    [ $rc -le 1 ] || exit $rc
    echo "== w43$v run $r: $(grep -h '^b' $O/w43${v}_$r.log | awk '{printf "%s %s  ", $1, $11}')"
  done
done
