#!/bin/bash
# GPU-box quick check: pytest -m gpu (one process) -> short bench without the
# CPU baseline.  Stops at the first GPU step that faults, aborts or times out.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "== pytest_gpu rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -3
if [ $rc -ne 0 ]; then tail -40 gpurun_out/pytest_gpu.log; exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc=$?
echo "== bench rc=$rc"; tail -3 gpurun_out/bench.log
exit $rc
