#!/bin/bash
# Round 5: POOL2 epilogue store ablation (SEDX_W43_ABL 32: every pooled store to one coalesced
# run, results WRONG) against the tree's kernel, B = 32: the most coalescing could give
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05zj
mkdir -p $O
for r in 1 2; do
  for v in "" _abl32; do
    timeout -k 10 200 tools/bin/w43_bench$v 32 20 > $O/w43${v}_$r.log 2>&1; rc=$?
    [ $rc -le 1 ] || exit $rc
    echo "variant '$v' round $r: $(grep -h '^b1c2\|^b2c2\|^b3c2\|^b4c2' $O/w43${v}_$r.log | awk '{printf "%s %s  ", $1, $11}')"
  done
done | tee $O/ab.txt
