#!/bin/bash
# Round 5: GRU slices spread over every XCD (SEDX_GRU_HANDOFF_SPREAD) beside the next batch's conv stack:
# handoff bit-identity test, then the headline A/B auto / spread / global, alternating
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05t
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -s --timeout 300 --timeout-method thread \
  -k "handoff or gru" > $O/pytest_gru.log 2>&1 || { tail -30 $O/pytest_gru.log; exit 1; }
grep -h "GRU hand-off\|passed" $O/pytest_gru.log
for r in 1 2; do
  for h in auto spread global; do
    timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-side --gru-handoff $h > $O/bench_${h}_$r.log 2>&1 || exit 1
    python3 - $O/bench_${h}_$r.log $h $r <<'PY'
import json, sys
ln = [l for l in open(sys.argv[1]) if l.startswith('{')][-1]
d = json.loads(ln)
st = d.get('stage_ms', {})
print(sys.argv[2], 'round', sys.argv[3], d['value'], d['ms_per_step'], {k: round(st[k], 3) for k in ('b1c1', 'b1c2', 'b2c1', 'b2c2', 'seq', 'head', 'frontend')})
PY
  done
done
