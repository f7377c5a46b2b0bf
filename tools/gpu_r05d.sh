#!/bin/bash
# Round 5: F(4,3) epilogue ablations (every MFMA live; exchange removed / barriers removed)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05d
mkdir -p $O
for v in abl4 abl8; do
  timeout -k 10 150 tools/bin/w43_bench_$v 32 10 > $O/w43_$v.log 2>&1; rc=$?
  [ $rc -le 1 ] || exit $rc
done
grep -h total $O/w43_abl*.log
