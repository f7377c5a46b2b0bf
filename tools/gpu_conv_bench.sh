#!/bin/bash
# Conv layer timing: current kernel, its s_memtime-stamped build, and (optionally)
# another revision of conv_x3.hip given as $CONV_PREV (path to a .hip file).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
HIPCC="/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -Xarch_device -mllvm=-disable-promote-alloca-to-lds"
C=sound-event-detection_amd/csrc
$HIPCC -o /tmp/cb_full tools/conv_bench.cpp $C/conv_x3.hip || exit 1
$HIPCC -DSEDX_CONV_STAMPS -o /tmp/cb_stamps tools/conv_bench.cpp $C/conv_x3.hip || exit 1
$HIPCC -DSEDX_CONV_ABL_NOSTORE -o /tmp/cb_nostore tools/conv_bench.cpp $C/conv_x3.hip || exit 1
for a in NOBAR NOLDS NOLOAD NOLOADA NOLOADW; do
  $HIPCC -DSEDX_ABL_$a -o /tmp/cb_$(echo $a | tr A-Z a-z) tools/conv_bench.cpp $C/conv_x3.hip || exit 1
done
$HIPCC -DSEDX_ABL_NOLDS -DSEDX_ABL_NOLOAD -o /tmp/cb_nostage tools/conv_bench.cpp $C/conv_x3.hip || exit 1
$HIPCC -DSEDX_ABL_NOLDS -DSEDX_ABL_NOLOAD -DSEDX_ABL_NOBAR -DSEDX_CONV_ABL_NOSTORE -o /tmp/cb_compute tools/conv_bench.cpp $C/conv_x3.hip || exit 1

if [ -n "$CONV_PREV" ]; then $HIPCC -o /tmp/cb_prev tools/conv_bench.cpp "$CONV_PREV" || exit 1; fi
for v in ${VARIANTS:-full stamps nostore full}; do
  [ -x /tmp/cb_$v ] || continue
  echo "== $v" | tee -a gpurun_out/conv_bench.log
  timeout -k 10 120 /tmp/cb_$v 32 20 | tee -a gpurun_out/conv_bench.log || exit $?
done
