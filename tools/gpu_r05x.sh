#!/bin/bash
# Round 5: the interleaved-halves GRU kernel (variant 5 / SEDX_GRU_KERNEL_PAIR): stamped micro-bench
# (bit-identity vs variant 0, ms per launch), GRU GPU tests, then p50 (one batch at a time) A/B auto vs pair
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05x
mkdir -p $O
for b in 32 256; do
  timeout -k 10 120 tools/bin/gru_bench $b 125 > $O/gru_bench_b$b.log 2>&1 || { cat $O/gru_bench_b$b.log; exit 1; }
  grep -h "differ\|us/step" $O/gru_bench_b$b.log | grep -v "v0 exact\|v1 exact\|v2 x3"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "gru" > $O/pytest_gru.log 2>&1 || { tail -30 $O/pytest_gru.log; exit 1; }
tail -1 $O/pytest_gru.log
