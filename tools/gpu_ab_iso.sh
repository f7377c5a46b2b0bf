#!/bin/bash
# A/B of package builds (tools/ab_build.sh) on the isolated (one batch at a
# time) per-stage times and the headline: full bench legs, alternating rounds.
#   VARIANTS="pre ..." bash tools/gpu_ab_iso.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  for v in tree ${VARIANTS}; do
    if [ $v = tree ]; then P=""; else P="--ab-package $PWD/sound-event-detection_amd/build/ab/$v"; fi
    timeout -k 10 300 python bench.py $P --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS} \
      > gpurun_out/abi_$v$r.log 2>&1 || exit $?
    python3 -c "
import json
s=open('gpurun_out/abi_$v$r.log').read(); d=json.loads(s[s.rfind('{\"metric\"'):].split('\n')[0])
iso=d['stage_ms_isolated']
print('$v round $r', d['value'], 'clips/s | iso', ' '.join('%s %.4f' % (k, v) for k, v in iso.items()))"
  done
done
