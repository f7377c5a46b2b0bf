#!/bin/bash
# GPU-box sequence: pytest -m gpu (one process, per-test timeout) -> profile_round.sh
# (full bench with CPU baseline, kernel-trace stats, FETCH_SIZE / WRITE_SIZE PMC passes).
# Stops at the first GPU step that faults, aborts or times out.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "== pytest_gpu rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -3
if [ $rc -ne 0 ]; then tail -40 gpurun_out/pytest_gpu.log; exit $rc; fi
bash tools/profile_round.sh
