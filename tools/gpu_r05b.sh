#!/bin/bash
# Round 5: chunk-of-4 layout for the F(4,3) chain — standalone check (C4 must
# equal NHWC bit for bit), winograd + new GPU tests, headline bench, and the
# 2-rank gloo rehearsal of the N > 1 path with the real model on one GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05b
mkdir -p $O
timeout -k 10 150 tools/bin/w43_bench 32 10 > $O/w43.log 2>&1; rc=$?
echo "w43 rc=$rc"; tail -n 2 $O/w43.log
[ $rc -eq 0 ] || exit 4
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -k "(wino and not x3) or spin_timeout_raises or stage_times or stage_goldens" > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -n 3 $O/tests.log
[ $rc -eq 0 ] || exit 5
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-side > $O/bench.log 2>&1 || exit 6
tail -c 400 $O/bench.log
timeout -k 10 400 python bench.py --gpus 2 --backend gloo --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_2rank.log 2>&1
echo "2rank rc=$?"; tail -c 300 $O/bench_2rank.log
