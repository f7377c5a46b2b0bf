#!/bin/bash
# rocprofv3 kernel stats of the frontend at several batch sizes (fixed vs per-frame cost)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for B in ${FE_BATCHES:-8 32 128}; do
  mkdir -p gpurun_out/feprof$B
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/feprof$B -o fe -- python tools/fe_bench.py $B 10 > gpurun_out/feprof$B/run.log 2>&1 || exit $?
  f=$(find gpurun_out/feprof$B -name "*kernel_stats.csv" | head -1); echo "B=$B"; grep -E "logmel|conv1_nhwc" "$f" | cut -d, -f1,4 | cut -c1-120
done
