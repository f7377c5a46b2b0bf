#!/bin/bash
# Winograd items-per-workgroup A/B: standalone layer times, then the headline bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
RUN=1 VARIANTS="${VARIANTS:-full i2 i8 i1000}" BATCHES=32 REPS=30 bash tools/gpu_wino.sh 2>&1 | grep -E "==|total" || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-side > gpurun_out/bench_ab.log 2>&1 || exit $?
python -c "import json; d=json.loads([l for l in open('gpurun_out/bench_ab.log') if l.startswith('{')][-1]); print('bench', d['value'], d['ms_per_step'], d.get('stage_ms'))"
