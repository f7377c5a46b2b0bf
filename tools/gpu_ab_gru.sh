#!/bin/bash
# A/B of the GRU kernel in the two-stream bench (headline only), alternating
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  for k in ${KERNELS:-coop tag16}; do
    timeout -k 10 240 python bench.py --steps 30 --warmup 5 --no-side --no-cpu-baseline --gru-kernel $k \
      > gpurun_out/ab_gru_${k}_${r}.json 2> gpurun_out/ab_gru_${k}_${r}.err || exit $?
    python -c "import json,sys; d=json.loads(open('gpurun_out/ab_gru_${k}_${r}.json').read().splitlines()[-1]); print('$k round $r', d['value'], 'p50', d['ms_per_clip_p50'], 'stage', d['stage_ms'])"
  done
done
