#!/bin/bash
# GPU-box check: pytest -m gpu (one process, per-test timeout) -> full bench
# (with the CPU baseline unless BENCH_ARGS says otherwise).  Stops at the
# first GPU step that faults, aborts or times out.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS} \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "== pytest_gpu rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -3
if [ $rc -ne 0 ]; then tail -60 gpurun_out/pytest_gpu.log; exit $rc; fi
timeout -k 10 600 python bench.py --steps 20 --warmup 3 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc=$?
echo "== bench rc=$rc"; tail -c 6000 gpurun_out/bench.log
exit $rc
