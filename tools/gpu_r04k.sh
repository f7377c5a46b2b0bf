#!/bin/bash
# Round 4: gamma frontend (first FFT stage from registers, sqrt-fma
# magnitudes) and the cost-chosen item rounds: GPU suite, gamma and
# headline kernel traces + FETCH passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04k
mkdir -p $OUT
step() {
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n ${TAILN:-2} "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping"; exit $rc; fi
}
step tests 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/
G="--no-cpu-baseline --no-side --streams 1 --mode gamma"
step kt_gamma 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_gamma -o kt -- python bench.py --steps 10 --warmup 2 $G
A="--no-cpu-baseline --no-side --streams 1"
step fetch 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o p -- python bench.py $A --steps 3 --warmup 1
step kt 150 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python bench.py $A --steps 10 --warmup 2
echo ALLDONE
