#!/bin/bash
# Round 4, first GPU call: the windowed-driver parity tests, a quick bench,
# and SQ counter passes over the headline's kernels (one stream, headline
# only) for the Winograd conv's time split: wave-parked (SQ_WAIT_ANY),
# issue-stalled (SQ_WAIT_INST_ANY), issuing (SQ_ACTIVE_INST_ANY), MFMA busy,
# VALU / LDS instruction counts and LDS bank conflicts.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04a
mkdir -p $OUT
step() {
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 3 "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping"; exit $rc; fi
}
# soft: test failures (rc 1) are recorded and the script goes on; any other
# status (abort, fault, time limit) stops it
soft() {
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 3 "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping"; exit $rc; fi
}
soft tests 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_events.py -k "windowed or driver or long or vote or sweep or events or spin or concurrent"
step bench 200 python bench.py --steps 20 --no-side --no-cpu-baseline
# the packed-FP32 corruption: the round-3 reproducer, then the pinned
# instruction sequence of its failing loop (tools/pk_seq_probe.cpp; built
# on the CPU side: BUILD=1 tools/gpu_pk_evidence.sh + hipcc of the probe)
step fe_race_pk 150 sound-event-detection_amd/build/tools/fe_race_pk 10 8
step pk_seq 300 sound-event-detection_amd/build/tools/pk_seq_probe -1 32
A="--no-cpu-baseline --no-side --streams 1 --steps 3 --warmup 1"
step sq1 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq1 -o p -- python bench.py $A
step sq2 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU --output-format csv -d $OUT/sq2 -o p -- python bench.py $A
step sq3 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_WAVES --output-format csv -d $OUT/sq3 -o p -- python bench.py $A
echo ALLDONE
