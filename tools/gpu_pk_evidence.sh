#!/bin/bash
# Evidence for the packed-FP32 ban (DESIGN §4 "Packed FP32 beside MFMA"):
# the same FFT frontend variant built WITH packed FP32 (hipcc defaults: the
# SLP vectoriser emits v_pk_add/mul/fma_f32) and WITHOUT
# (-fno-slp-vectorize -fno-vectorize), each run beside an MFMA-only
# co-runner on a second stream and compared bit for bit with a serial run;
# then the minimal probes of tools/mfma_corun.cpp (probe 3: packed FP32
# chains, no LDS / memory; probes 0-2: scalar VALU, transcendental, LDS).
# Build here (BUILD=1), run on the GPU box (RUN=1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=sound-event-detection_amd/build/tools
mkdir -p $D gpurun_out
if [ -n "$BUILD" ]; then
  H="/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -w -Xarch_device -mllvm=-disable-promote-alloca-to-lds"
  S="tools/fe_race.cpp sound-event-detection_amd/csrc/frontend.hip sound-event-detection_amd/csrc/linear_x3.hip sound-event-detection_amd/csrc/conv_x3.hip"
  $H -o $D/fe_race_pk $S || exit 1
  $H -fno-slp-vectorize -fno-vectorize -o $D/fe_race_nopk $S || exit 1
  $H -o $D/mfma_corun tools/mfma_corun.cpp || exit 1
  for v in pk nopk; do
    f=""; [ $v = nopk ] && f="-fno-slp-vectorize -fno-vectorize"
    $H $f --cuda-device-only -S -o $D/fe_race_$v.s tools/fe_race.cpp || exit 1
  done
fi
[ -n "$RUN" ] || exit 0
for v in pk nopk; do
  echo "== fe_race_$v: $(grep -cE 'v_pk_(add|mul|fma)_f32' $D/fe_race_$v.s) packed-FP32 instructions in its device code"
  timeout -k 10 120 $D/fe_race_$v 10 8 || exit $?    # variant 0 beside the MFMA co-runner, 8 rounds
done
timeout -k 10 180 $D/mfma_corun 8 || exit $?
