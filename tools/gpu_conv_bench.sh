#!/bin/bash
# x3 conv layer timing: the current kernel and its s_memtime-stamped build
# (phase split), optionally another revision of conv_x3.hip ($CONV_PREV).
# Build here on the CPU (BUILD=1, binaries in tools/prev/), run on the box (RUN=1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out tools/prev
HIPCC="/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fno-slp-vectorize -fno-vectorize -Xarch_device -mllvm=-disable-promote-alloca-to-lds -Isound-event-detection_amd/csrc"
C=sound-event-detection_amd/csrc
O=tools/prev
if [ -n "$BUILD" ]; then
  $HIPCC -o $O/cb_full tools/conv_bench.cpp $C/conv_x3.hip || exit 1
  $HIPCC -DSEDX_CONV_STAMPS -o $O/cb_stamps tools/conv_bench.cpp $C/conv_x3.hip || exit 1
  if [ -n "$CONV_PREV" ]; then $HIPCC -o $O/cb_prev tools/conv_bench.cpp "$CONV_PREV" || exit 1; fi
fi
[ -n "$RUN" ] || exit 0
for v in ${VARIANTS:-full stamps}; do
  [ -x $O/cb_$v ] || continue
  echo "== $v" | tee -a gpurun_out/conv_bench.log
  timeout -k 10 120 $O/cb_$v 32 20 | tee -a gpurun_out/conv_bench.log || exit $?
done
