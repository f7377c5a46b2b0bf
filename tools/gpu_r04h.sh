#!/bin/bash
# Round 4: the K-split GRU hand-off (SEDX_GRU_KERNEL_KSPLIT) — micro-bench
# with per-phase stamps (every exact variant's bits compared), the GRU GPU
# tests, and the p50 / headline with each kernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04h
mkdir -p $OUT
step() {
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n ${TAILN:-12} "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping"; exit $rc; fi
}
step gru32 120 sound-event-detection_amd/build/tools/gru_bench 32 125
step gru256 120 sound-event-detection_amd/build/tools/gru_bench 256 125
TAILN=3 step tests 400 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "gru"
A="--steps 30 --no-side --no-cpu-baseline"
for r in 1 2; do
  for k in auto ksplit; do TAILN=1 step bench_${k}_$r 300 python bench.py $A --gru-kernel $k; done
done
echo ALLDONE
