#!/bin/bash
# Exact conv layer timing + SQ counters.  BUILD=1 (here, CPU): binaries into
# tools/prev/ from the current conv.hip and every tools/prev/conv_*.hip
# variant; RUN=1 (GPU box): time each, then one SQ-counter pass of cx_full.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out tools/prev
HIPCC="/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -Wno-unused-result -Wno-unused-value -fno-slp-vectorize -fno-vectorize -Isound-event-detection_amd/csrc"
C=sound-event-detection_amd/csrc
O=tools/prev
if [ -n "$BUILD" ]; then
  $HIPCC -o $O/cx_full tools/conv_exact_bench.cpp $C/conv.hip || exit 1
  $HIPCC -DSEDX_EXACT_STAMPS -o $O/cx_stamps tools/conv_exact_bench.cpp $C/conv.hip || exit 1
  for v in $O/conv_*.hip; do
    [ -f "$v" ] || continue
    n=$(basename $v .hip); n=${n#conv_}
    sed "s/launch_block1_exact(in, B, l.T, w1, b1, w, bias, out, zero, 0)/launch_block1_exact(in, B, l.T, w1, b1, w, bias, out, 0)/; s/l.epi, zero, 0)/l.epi, 0)/" tools/conv_exact_bench.cpp > tools/prev/cxb_old.cpp; if grep -q zero16 $v; then $HIPCC -o $O/cx_$n tools/conv_exact_bench.cpp $v || exit 1; else $HIPCC -Itools -o $O/cx_$n tools/prev/cxb_old.cpp $v || exit 1; fi
  done
fi
[ -n "$RUN" ] || exit 0
export TMPDIR=/tmp
for v in ${VARIANTS:-full}; do
  echo "== $v" | tee -a gpurun_out/conv_exact.log
  for bb in ${BATCHES:-32}; do timeout -k 10 120 $O/cx_$v $bb 20 || exit $?; done | tee -a gpurun_out/conv_exact.log || exit $?
done
if [ -n "$PMC" ]; then
  timeout -k 10 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_MFMA GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/cx_pmc -o p -- $O/cx_full 32 5 > gpurun_out/cx_pmc.log 2>&1 || exit $?
  timeout -k 10 180 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/cx_pmc2 -o p -- $O/cx_full 32 5 > gpurun_out/cx_pmc2.log 2>&1 || exit $?
fi
echo done
