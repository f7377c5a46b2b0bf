#!/bin/bash
# Headline-leg A/B on one GPU box: bench.py --no-side --no-cpu-baseline with
# each argument set in turn (separated by '|', ',' reads as ' '), ROUNDS
# alternating rounds; prints value / ms_per_step / seq / b1c2 per run.
#   tools/ab_headline.sh TAG "--wino-order,1|--wino-order,2" [ROUNDS]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:?tag}; IFS='|' read -r -a SETS <<< "${2:?arg sets}"; R=${3:-2}
O=gpurun_out/$TAG
mkdir -p "$O"
for r in $(seq 1 "$R"); do
  i=0
  for a in "${SETS[@]}"; do
    i=$((i + 1))
    f=$O/ab_r${r}_s$i.log
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-side --no-cpu-baseline ${a//,/ } > "$f" 2>&1 \
      || { echo "run $r set $i failed"; tail -5 "$f"; exit 1; }
    python - "$f" "$a" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d = json.loads(l); st = d.get('stage_ms') or {}
        print('%-28s %9.1f clips/s  %.4f ms/step  seq %.3f  b1c2 %.3f  b2c1 %.3f' % (
            sys.argv[2], d['value'], d['ms_per_step'], st.get('seq', 0), st.get('b1c2', 0), st.get('b2c1', 0)))
PY
  done
done
