#!/bin/bash
# Winograd conv check + timing (tools/wino_bench.cpp).  BUILD=1 (here, CPU):
# tools/prev/wb_full from the tree's conv.hip + conv_wino.hip; RUN=1 (GPU
# box): run it at each of BATCHES (default 32 4 1), optional PMC pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out tools/prev
HIPCC="/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -Wno-unused-result -Wno-unused-value -fno-slp-vectorize -fno-vectorize -Isound-event-detection_amd/csrc"
C=sound-event-detection_amd/csrc
O=tools/prev
if [ -n "$BUILD" ]; then
  $HIPCC -o $O/wb_full tools/wino_bench.cpp $C/conv.hip $C/conv_wino.hip || exit 1
  # VARIANT_FLAGS: "name:-DFLAG=1,-DOTHER name2:..." extra builds
  for vf in $VARIANT_FLAGS; do n=${vf%%:*}; f=${vf#*:}; $HIPCC ${f//,/ } -o $O/wb_$n tools/wino_bench.cpp $C/conv.hip $C/conv_wino.hip || exit 1; done
  for nb in $NBUFS; do $HIPCC -DSEDX_WINO_NBUF=$nb -o $O/wb_nb$nb tools/wino_bench.cpp $C/conv.hip $C/conv_wino.hip || exit 1; done
fi
[ -n "$RUN" ] || exit 0
export TMPDIR=/tmp
for v in ${VARIANTS:-full}; do
  echo "== $v"
  for bb in ${BATCHES:-32 4 1}; do
    timeout -k 10 300 $O/wb_$v $bb ${REPS:-20}; rc=$?; [ $rc -le 1 ] || exit $rc   # 1 = mismatch (ablations)
  done
done 2>&1 | tee -a gpurun_out/wino.log || exit $?
if [ -n "$PMC" ]; then
  timeout -k 10 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/wb_pmc -o p -- $O/wb_full 32 3 > gpurun_out/wb_pmc.log 2>&1 || exit $?
  timeout -k 10 180 rocprofv3 --pmc FETCH_SIZE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/wb_pmc2 -o p -- $O/wb_full 32 3 > gpurun_out/wb_pmc2.log 2>&1 || exit $?
fi
echo done
