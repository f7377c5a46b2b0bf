#!/bin/bash
# Round 5: persistent F(4,3) workgroups (SEDX_W43_ITEMS 16): check, winograd GPU tests, headline
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05o
mkdir -p $O
timeout -k 10 200 tools/bin/w43_bench 32 10 > $O/w43.log 2>&1; rc=$?
grep -h "total" $O/w43.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "wino or winograd or stage or batch32 or driver_windows or golden" > $O/pytest_wino.log 2>&1 || { tail -30 $O/pytest_wino.log; exit 1; }
tail -1 $O/pytest_wino.log
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-side > $O/bench_$r.log 2>&1 || exit 1
  grep -o '"value": [0-9.]*' $O/bench_$r.log | head -1
done
