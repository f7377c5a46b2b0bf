#!/bin/bash
# Round 4, third GPU call: the Transformer tests after the XCD-aware MHA grid,
# the operand-select variants of the packed-FP32 probe (10-15), and the
# config-3 (Transformer) profile: kernel trace + FETCH / WRITE + MFMA passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04c
mkdir -p $OUT
step() {
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 3 "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping"; exit $rc; fi
}
step tests 400 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "transformer or config5 or mha"
for v in 10 11 12 13 14 15; do
  step pk_seq_$v 120 sound-event-detection_amd/build/tools/pk_seq_probe $v 16
done
NO_FULL=1 PRECISIONS=" " LEGS=config3 timeout -k 10 900 bash tools/profile_round.sh > $OUT/prof_config3.log 2>&1 || exit $?
echo ALLDONE
