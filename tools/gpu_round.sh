#!/bin/bash
# GPU-box sequence: smoke -> pytest -m gpu -> short bench.  Stops on any
# fault/abort/timeout (exit codes other than 0 and 1); a plain test failure
# (exit 1) still lets the bench run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
run smoke 300 python -c "import __graft_entry__ as g; g.build(); g.smoke()"
run pytest_gpu 900 python -m pytest tests -m gpu -x -q -s
run bench 600 python bench.py --steps ${BENCH_STEPS:-10} --warmup 3 ${BENCH_ARGS}
