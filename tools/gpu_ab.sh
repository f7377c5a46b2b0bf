#!/bin/bash
# GPU box: parity tests of the current build, then an A/B of conv-layer
# timings (tools/prev/cb_*: built here on the CPU, VARIANTS in run order),
# then a short bench.  Stops at the first step that fails.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "== pytest_gpu rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
  [ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_gpu.log; exit $rc; }
fi
for v in ${VARIANTS:-prev nogw full prev nogw full}; do
  echo "== $v" >> gpurun_out/conv_ab.log
  timeout -k 10 120 tools/prev/cb_$v 32 20 >> gpurun_out/conv_ab.log 2>&1 || { echo "cb_$v failed"; tail gpurun_out/conv_ab.log; exit 1; }
done
grep -E "^==|total" gpurun_out/conv_ab.log
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-exact ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc=$?; echo "== bench rc=$rc"; tail -c 600 gpurun_out/bench.log
exit $rc
