#!/bin/bash
# Round 5: default bench on the final tree with the r05zl profile in the roofline
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05zm
mkdir -p $O
timeout -k 10 900 python -u bench.py > $O/bench_full.log 2>&1 || { tail -20 $O/bench_full.log; exit 1; }
grep -o '"value": [0-9.]*' $O/bench_full.log | head -1
