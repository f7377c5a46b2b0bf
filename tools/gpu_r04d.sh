#!/bin/bash
# Round 4: wino_block1_kernel's time split.
# BUILD=1 (here, CPU): the stand-alone bench tools/wino_b1_bench.cpp as a plain
# build, an s_memtime-stamped build (SEDX_WINO_STAMPS) and five ablation builds
# (SEDX_WINO_ABL 1 conv1, 2 transform, 4 patch LDS reads, 8 U LDS reads, 16
# chunk DMAs: wrong outputs, timing only).  On the box: each binary once,
# plain first and last (run-to-run noise).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=sound-event-detection_amd/build/tools
C=sound-event-detection_amd/csrc
if [ -n "$BUILD" ]; then
  H="/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fno-slp-vectorize -fno-vectorize"
  mkdir -p $O
  $H -o $O/wb1_plain tools/wino_b1_bench.cpp $C/conv_wino.hip || exit 1
  $H -DSEDX_WINO_STAMPS -o $O/wb1_stamps tools/wino_b1_bench.cpp $C/conv_wino.hip || exit 1
  for a in 1 2 4 8 16; do $H -DSEDX_WINO_ABL=$a -o $O/wb1_abl$a tools/wino_b1_bench.cpp $C/conv_wino.hip || exit 1; done
  exit 0
fi
OUT=gpurun_out/r04d
mkdir -p $OUT
step() {
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 12 "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping"; exit $rc; fi
}
step plain0 120 $O/wb1_plain 32 20 plain
step stamps 120 $O/wb1_stamps 32 20 stamps
for a in 1 2 4 8 16; do step abl$a 120 $O/wb1_abl$a 32 20 abl$a any; done
step plain1 120 $O/wb1_plain 32 20 plain
echo ALLDONE
