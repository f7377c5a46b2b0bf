#!/bin/bash
# Round 5: F(4,3) check after the per-EPI exchange layouts, then the full GPU test suite and smoke()
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05l
mkdir -p $O
timeout -k 10 200 tools/bin/w43_bench 32 10 > $O/w43.log 2>&1; rc=$?
grep -h "^b\|total" $O/w43.log | cut -c1-80
[ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
