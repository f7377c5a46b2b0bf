#!/bin/bash
# Round 4: (1) the gammatone frontend after the ERB kernel's register-direct
# magnitudes and the first FFT stage from registers — gamma tests, config-4
# leg with kernel trace; (2) the L2-friendly item order on 64-channel groups
# (8 tile blocks x 4 groups per round) — parity test, FETCH_SIZE and kernel
# trace per order, alternating headline rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04j
mkdir -p $OUT
step() {
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "stopping"; exit $rc; fi
}
step tests 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/ -k "gamma or wino_order or config4"
G="--no-cpu-baseline --no-side --streams 1 --mode gamma"
step kt_gamma 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_gamma -o kt -- python bench.py --steps 10 --warmup 2 $G
step fetch_gamma 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch_gamma -o p -- python bench.py --steps 3 --warmup 1 $G
step mfma_gamma 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/mfma_gamma -o p -- python bench.py --steps 3 --warmup 1 $G
A="--no-cpu-baseline --no-side --streams 1 --steps 3 --warmup 1"
for o in 0 1; do
  step fetch_o$o 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch_o$o -o p -- python bench.py $A --wino-order $o
  step kt_o$o 150 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_o$o -o kt -- python bench.py --no-cpu-baseline --no-side --streams 1 --steps 10 --warmup 2 --wino-order $o
done
for r in 1 2; do
  for o in 0 1; do
    TAILN=1 step bench_o${o}_r$r 200 python bench.py --steps 30 --no-side --no-cpu-baseline --wino-order $o
  done
done
echo ALLDONE
