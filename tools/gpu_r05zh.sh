#!/bin/bash
# Round 5: F(4,3) STORE finisher with each kc's 16 lanes on 16 consecutive pixels (256-byte runs):
# w43_bench B = 32 / 1 (checks against the direct reference + times), winograd parity tests,
# then the headline leg
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05zh
mkdir -p $O
for b in 32 1; do
  timeout -k 10 200 tools/bin/w43_bench $b 20 > $O/w43_b$b.log 2>&1; rc=$?
  [ $rc -le 1 ] || exit $rc
  grep -h "^b2c1\|^b3c1\|^b4c1\|^total" $O/w43_b$b.log | cut -c1-150
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "invariance or small_batch or multi_clip or wino or winograd or batch32" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-side > $O/bench_$r.log 2>&1 || { tail -20 $O/bench_$r.log; exit 1; }
  echo "bench round $r: $(grep -o '"value": [0-9.]*' $O/bench_$r.log | head -1)"
done
