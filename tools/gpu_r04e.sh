#!/bin/bash
# Round 4: the row-wave Winograd layout (4 waves per tile group, 64 channels
# per wave) against round 3's wave-pair layout: stand-alone layers (outputs
# vs the direct conv and float64; time), block 1, B = 1 shapes, the GPU test
# suite, and the headline A/B against the round-3 build (tools/ab_build.sh old).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04e
O=sound-event-detection_amd/build/tools
mkdir -p $OUT
step() {
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n ${TAILN:-9} "$OUT/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "stopping"; exit $rc; fi
}
step wb_old 120 $O/wb_old 32 20
step wb_new 120 $O/wb_new 32 20
step wb1_old 120 $O/wb1_old 32 20 old
step wb1_new 120 $O/wb1_new 32 20 new
step wb_new_b1 120 $O/wb_new 1 20
step wb_old_b1 120 $O/wb_old 1 20
TAILN=4 step tests 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/
A="--steps 30 --no-side --no-cpu-baseline"
for r in 1 2; do
  TAILN=1 step bench_new_$r 300 python bench.py $A
  TAILN=1 step bench_old_$r 300 python bench.py $A --ab-package sound-event-detection_amd/build/ab/old
done
echo ALLDONE
