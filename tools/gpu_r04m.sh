#!/bin/bash
# Round 4: the one-wave-per-frame gammatone spectrum (SEDX_TUNE_GAMMA_SPEC 1):
# codes vs the oracle with both kernels, config-4 kernel trace per kernel,
# config-4 leg A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04m
mkdir -p $OUT
step() {
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n ${TAILN:-2} "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping"; exit $rc; fi
}
step tests 300 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "gamma"
G="--no-cpu-baseline --no-side --streams 1 --mode gamma"
for v in 0 1; do
  step kt_gs$v 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_gs$v -o kt -- python bench.py --steps 10 --warmup 2 $G --gamma-spec $v
done
echo ALLDONE
