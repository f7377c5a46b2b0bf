#!/bin/bash
# Round 5: small-batch F(2,3) vs F(4,3) per layer (B = 1, 2, 4, 8)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05q2
mkdir -p $O
for b in 1 2 4 8 32; do
  timeout -k 10 200 tools/bin/w43_bench $b 20 > $O/w43_b$b.log 2>&1; rc=$?
  [ $rc -le 1 ] || exit $rc
  echo "== B=$b: $(grep -h '^b' $O/w43_b$b.log | awk '{printf "%s %s/%s  ", $1, $5, $11}')"
  grep -h "^block1\|^total" $O/w43_b$b.log | cut -c1-160
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "invariance or small_batch or multi_clip or wino or winograd or batch32" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
