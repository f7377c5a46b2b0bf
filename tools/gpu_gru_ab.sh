#!/bin/bash
# GRU recurrence kernels in the headline: throughput, p50 and the seq stage
# (two-stream timed region and one batch at a time) per SEDX_TUNE_GRU_KERNEL.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in ${ROUNDS:-1 2}; do
  for k in ${KERNELS:-coop tag16 tag8 coop16}; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS} --gru-kernel $k > gpurun_out/gru_$k$r.log 2>&1 || exit $?
    python3 -c "
import json
s=open('gpurun_out/gru_$k$r.log').read(); d=json.loads(s[s.rfind('{\"metric\"'):].split('\n')[0])
st=d['stage_ms']; iso=d.get('stage_ms_isolated') or {}
print('$k round $r', d['value'], 'clips/s p50', d['ms_per_clip_p50'], '| seq timed', st.get('seq'), 'iso', iso.get('seq'), '| b1c2 timed', st.get('b1c2'), 'iso', iso.get('b1c2'), '| conv iso', round(sum(v for k_, v in iso.items() if k_[0] == 'b'), 4))"
  done
done
