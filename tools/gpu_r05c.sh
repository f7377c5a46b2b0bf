#!/bin/bash
# Round 5: F(4,3) tweaks (no item-top barrier, wave 11's halo DMA into a trash
# block, per-channel-tile stores) — standalone check + ablations, winograd GPU
# tests, headline bench; then the round's profiles (winograd headline,
# config 3, config 4, window mode).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05c
mkdir -p $O
timeout -k 10 150 tools/bin/w43_bench 32 10 > $O/w43.log 2>&1; rc=$?
echo "w43 rc=$rc"; tail -n 1 $O/w43.log
[ $rc -eq 0 ] || exit 4
for v in abl1 abl2 abl4; do
  timeout -k 10 150 tools/bin/w43_bench_$v 32 10 > $O/w43_$v.log 2>&1; rc=$?
  [ $rc -le 1 ] || exit $rc
done
grep -h total $O/w43_abl*.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -k "(wino and not x3) or spin_timeout_raises or stage_times or stage_goldens" > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -n 2 $O/tests.log
[ $rc -eq 0 ] || exit 5
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-side > $O/bench.log 2>&1 || exit 6
tail -c 300 $O/bench.log; echo
NO_FULL=1 PRECISIONS=winograd LEGS="config3 config4 window" bash tools/profile_round.sh
