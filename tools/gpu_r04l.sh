#!/bin/bash
# Round 4: block 1's conv1 on the matrix pipe (v_mfma_f32_4x4x1f32): the
# 4x4x1 layout / fma-chain probe, then the stand-alone block-1 kernel with
# VALU and MFMA conv1 (output hashes must match: same bits), two rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04l
O=sound-event-detection_amd/build/tools
mkdir -p $OUT
step() {
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping"; exit $rc; fi
}
step probe 60 $O/mfma4x4_probe
for r in 1 2; do
  for v in new c1m c1m4; do step wb1_${v}_$r 120 $O/wb1_$v 32 20 $v; done
done
echo ALLDONE
