#!/bin/bash
# Round 5: SQ counter split of the F(4,3) conv kernels (headline, one stream) — sq_summary.py input
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05k
mkdir -p $OUT
A="--no-cpu-baseline --no-side --streams 1 --steps 3 --warmup 1"
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq1 -o p -- python bench.py $A > $OUT/sq1.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU --output-format csv -d $OUT/sq2 -o p -- python bench.py $A > $OUT/sq2.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_WAVES --output-format csv -d $OUT/sq3 -o p -- python bench.py $A > $OUT/sq3.log 2>&1 || exit 1
echo ALLDONE
