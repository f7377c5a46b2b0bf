#!/bin/bash
# Round 4: row-wave Winograd with 32 channels per wave and 3 or 4 waves per
# SIMD (12 / 16-wave workgroups) against the 64-channel, 2-wave default;
# stand-alone blocks 2-4, three alternating rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04g
O=sound-event-detection_amd/build/tools
mkdir -p $OUT
step() {
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -E "total|MISMATCH" "$OUT/$name.log" | cut -c1-200
  if [ $rc -ne 0 ]; then echo "stopping"; exit $rc; fi
}
for r in 1 2 3; do
  for v in new tg3 tg4; do step wb_${v}_$r 120 $O/wb_$v 32 20; done
done
echo ALLDONE
