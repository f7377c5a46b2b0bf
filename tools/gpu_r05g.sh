#!/bin/bash
# Round 5: F(4,3) block 1 (default WINO_F43 2): winograd GPU tests + headline A/B against F43 1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05g
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "wino or winograd or stage or batch32 or driver_windows or golden" > $O/pytest_wino.log 2>&1 || { tail -30 $O/pytest_wino.log; exit 1; }
tail -3 $O/pytest_wino.log
for f in 2 1 2 1; do
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-side --wino-f43 $f > $O/bench_f43_$f.log 2>&1 || exit 1
  python - $O/bench_f43_$f.log <<'PY'
import json, sys
ln = [l for l in open(sys.argv[1]) if l.startswith('{')][-1]
d = json.loads(ln)
print(sys.argv[1], d['value'], d['ms_per_step'], {k: round(v, 3) for k, v in d.get('stage_ms', {}).items() if k.startswith('b')})
PY
done
