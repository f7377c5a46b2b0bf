#!/bin/bash
# Winograd change check: standalone layer times (B 32 / 4), Winograd parity subset, headline bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
RUN=1 VARIANTS="full" BATCHES="32 4" REPS=30 bash tools/gpu_wino.sh 2>&1 | grep -E "==|wino|total" | cut -c1-75 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "wino or small_batch or stage_goldens or past_32bit or long_clip" > gpurun_out/t_w.log 2>&1; rc=$?; grep -E "passed|failed" gpurun_out/t_w.log | tail -2; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-side > gpurun_out/bench_ab.log 2>&1 || exit $?
python -c "import json; d=json.loads([l for l in open('gpurun_out/bench_ab.log') if l.startswith('{')][-1]); print('bench', d['value'], d['ms_per_step'], d.get('stage_ms'))"
