#!/bin/bash
# Round 5: pipelined headline with the GRU slices spread: 8-slice (auto) vs 16-slice (coop16) vs K-split, alternating
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05za
mkdir -p $O
for r in 1 2; do
  for k in auto coop16 ksplit; do
    timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-side --gru-kernel $k > $O/bench_${k}_$r.log 2>&1 || exit 1
    python3 - $O/bench_${k}_$r.log $k $r <<'PY'
import json, sys
ln = [l for l in open(sys.argv[1]) if l.startswith('{')][-1]
d = json.loads(ln)
st = d.get('stage_ms', {})
print(sys.argv[2], 'round', sys.argv[3], d['value'], d['ms_per_step'], {k: round(st[k], 3) for k in ('b1c2', 'b2c1', 'b2c2', 'seq', 'head', 'frontend')})
PY
  done
done
