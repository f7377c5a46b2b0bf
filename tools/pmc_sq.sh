#!/bin/bash
# SQ-level counters for the conv kernels (separate pass, kernel-trace only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/sq
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $OUT/a -o p -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-exact ${BENCH_ARGS} > $OUT/a.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_SALU --output-format csv -d $OUT/b -o p -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-exact ${BENCH_ARGS} > $OUT/b.log 2>&1 || exit $?
echo done
