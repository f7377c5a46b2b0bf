#!/bin/bash
# Round 4, second GPU call: the packed-FP32 single-instruction probes; the
# Winograd item-order A/B (SEDX_TUNE_WINO_ORDER: parity test, alternating
# headline rounds, FETCH_SIZE of the 512-channel layers per order).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04b
mkdir -p $OUT
step() {
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 4 "$OUT/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "stopping"; exit $rc; fi
}
step pk_seq 300 sound-event-detection_amd/build/tools/pk_seq_probe -1 16
step order_test 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "wino_order"
for r in 1 2; do
  for o in 0 1; do
    step bench_o${o}_r$r 200 python bench.py --steps 30 --no-side --no-cpu-baseline --wino-order $o
  done
done
A="--no-cpu-baseline --no-side --streams 1 --steps 3 --warmup 1"
for o in 0 1; do
  step fetch_o$o 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch_o$o -o p -- python bench.py $A --wino-order $o
  step kt_o$o 150 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_o$o -o kt -- python bench.py --no-cpu-baseline --no-side --streams 1 --steps 10 --warmup 2 --wino-order $o
done
echo ALLDONE
