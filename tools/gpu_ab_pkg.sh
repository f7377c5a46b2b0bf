#!/bin/bash
# A/B of the headline between the tree's build (B) and variant packages built
# by tools/ab_build.sh (bench.py --ab-package), alternating rounds in one GPU call.
#   VARIANTS="nb4 ..." bash tools/gpu_ab_pkg.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in ${ROUNDS:-1 2}; do
  for v in tree ${VARIANTS}; do
    if [ $v = tree ]; then P=""; else P="--ab-package $PWD/sound-event-detection_amd/${AB_ROOT:-build/ab}/$v"; fi
    timeout -k 10 300 python bench.py $P --steps ${STEPS:-30} --warmup 3 --no-cpu-baseline ${BENCH_ARGS:---no-side} \
      > gpurun_out/abp_$v$r.log 2>&1 || exit $?
    python3 -c "
import json
s=open('gpurun_out/abp_$v$r.log').read(); d=json.loads(s[s.rfind('{\"metric\"'):].split('\n')[0])
print('$v round $r', d['value'], 'clips/s', d['ms_per_step'], 'ms/step', d['library'], 'stage', d['stage_ms'])"
  done
done
