#!/bin/bash
# A/B of the headline between two builds of the package in one GPU call:
# A = tools/prev/pkg_old (bench.py --ab-package), B = the tree's build; alternating rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in ${ROUNDS:-1 2}; do
  for v in A B; do
    if [ $v = A ]; then P="--ab-package $PWD/tools/prev/pkg_old"; else P=""; fi
    timeout -k 10 300 python bench.py $P --steps ${STEPS:-30} --warmup 3 --no-side --no-cpu-baseline ${BENCH_ARGS} \
      > gpurun_out/ab_$v$r.log 2>&1 || exit $?
    python3 -c "
import json,sys
s=open('gpurun_out/ab_$v$r.log').read(); d=json.loads(s[s.rfind('{\"metric\"'):].split('\n')[0])
print('$v round $r', d['value'], 'clips/s', d['ms_per_step'], 'ms/step', 'b1c2 frac', d['roofline']['frac'], d['stage_ms'])"
  done
done
