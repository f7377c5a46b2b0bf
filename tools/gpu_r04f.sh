#!/bin/bash
# Round 4: tuning builds of the row-wave Winograd layout (ring depth 4, VALU
# group per MFMA 2 / 4, ~2 items per workgroup), two alternating rounds of
# the stand-alone layers; block 1's stamps + ablations in the new layout; SQ
# counter passes over the headline's launches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04f
O=sound-event-detection_amd/build/tools
mkdir -p $OUT
step() {
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n ${TAILN:-1} "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping"; exit $rc; fi
}
for r in 1 2; do
  for v in new nb4 vg2 vg4 it2; do
    step wb_${v}_$r 120 $O/wb_$v 32 20
    step wb1_${v}_$r 120 $O/wb1_$v 32 20 $v
  done
done
TAILN=12 step wb1_stamps 120 $O/wb1_stampsn 32 20 stamps
for a in 1 2 4 16; do step wb1_abl$a 120 $O/wb1_abln$a 32 20 abl$a any; done
A="--no-cpu-baseline --no-side --streams 1 --steps 3 --warmup 1"
step sq1 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq1 -o p -- python bench.py $A
step sq2 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU --output-format csv -d $OUT/sq2 -o p -- python bench.py $A
step kt 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python bench.py --steps 10 --warmup 2 $A
echo ALLDONE
