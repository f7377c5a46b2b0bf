#!/bin/bash
# GPU-box sequence used during development: optional GRU micro-bench, the GPU
# tests, then the bench.  Every step has its own time limit; the sequence
# stops at the first failing step (a fault, abort or time limit ends it).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
set -o pipefail
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 30 "gpurun_out/$name.log"
  return $rc
}
if [ -n "$GRU" ]; then
  for b in ${GRU_BATCHES:-32 256}; do
    step gru_bench_$b 120 sound-event-detection_amd/build/tools/gru_bench $b 125 || exit $?
  done
fi
if [ -z "$NOTEST" ]; then
  if [ -n "$PYTEST_K" ]; then
    step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$PYTEST_K" || exit $?
  else
    step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread || exit $?
  fi
fi
if [ -z "$NOBENCH" ]; then
  step bench 900 python bench.py --steps ${BENCH_STEPS:-20} --warmup 3 ${BENCH_ARGS} || exit $?
fi
