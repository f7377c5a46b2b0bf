#!/bin/bash
# scratch A/B of bench flags (one GPU call)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
i=0
for a in "--streams 2" "--streams 3" "--streams 1" "--streams 2 --no-pipeline"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-side $a > gpurun_out/ab_$i.log 2>&1 || exit $?
  python -c "import json; d=json.loads([l for l in open('gpurun_out/ab_$i.log') if l.startswith('{')][-1]); print('$a', d['value'], d['ms_per_step'])"
done
