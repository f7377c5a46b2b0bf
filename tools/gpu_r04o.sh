#!/bin/bash
# Round 4: Winograd items per workgroup in the two-stream headline (row-wave
# layout): default (~4, block 1 ~8) vs ~2 vs ~8 (block 1 ~16), three
# alternating rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04o
mkdir -p $OUT
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -o '"value": [0-9.]*' $OUT/$name.log | head -1)"
  if [ $rc -ne 0 ]; then echo "stopping"; exit $rc; fi
}
A="--steps 30 --no-side --no-cpu-baseline"
for r in 1 2 3; do
  step def_$r 200 python bench.py $A
  step it2_$r 200 python bench.py $A --ab-package sound-event-detection_amd/build/ab/it2
  step it8_$r 200 python bench.py $A --ab-package sound-event-detection_amd/build/ab/it8
done
echo ALLDONE
