#!/bin/bash
# GPU-box check for frontend / block-1 work: parity subset, frontend timing,
# headline bench with Winograd block 1 on and off.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "${PYTEST_K:-stage_goldens or short_clip or clip_goldens or batch32 or long_clip or windowed or int16 or batch_invariance or small_batch or winograd}" \
  > gpurun_out/fe_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|Error|assert" gpurun_out/fe_tests.log | tail -15
[ $rc -eq 0 ] || exit $rc
for wb in 1 0; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-side --wino-block1 $wb > gpurun_out/bench_wb$wb.log 2>&1 || exit $?
  python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/bench_wb$wb.log') if l.startswith('{')][-1]); print('wino_block1=$wb', d['value'], d['ms_per_step'], d.get('stage_ms'))"
done
