#!/bin/bash
# Round 4: full GPU suite, the round's profiles (kernel trace + FETCH / WRITE
# / MFMA passes) of the headline (winograd) and config 4, and a full bench run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04i
mkdir -p $OUT
step() {
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping"; exit $rc; fi
}
step tests 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/
NO_FULL=1 PRECISIONS="winograd" LEGS="config4" timeout -k 10 1000 bash tools/profile_round.sh > $OUT/prof.log 2>&1 || exit $?
TAILN=1 step bench_full 600 python bench.py
echo ALLDONE
