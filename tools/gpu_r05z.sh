#!/bin/bash
# Round 5: s_setprio around the F(4,3) MFMA groups (experiment), alternating
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05z
mkdir -p $O
for r in 1 2; do
  for v in "" _prio1 _prio3; do
    timeout -k 10 200 tools/bin/w43_bench$v 32 10 > $O/w43${v}_$r.log 2>&1; rc=$?
    [ $rc -le 1 ] || exit $rc
    echo "== w43$v run $r: $(grep -h '^b' $O/w43${v}_$r.log | awk '{printf "%s %s  ", $1, $11}') $(grep -h '^total' $O/w43${v}_$r.log | cut -c1-90)"
  done
done
