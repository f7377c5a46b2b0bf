#!/bin/bash
# Round 5: block 1 on F(4,3) (conv1 launch in the chunk-of-4 layout + F(4,3) conv2) vs the fused F(2,3) launch
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05f
mkdir -p $O
timeout -k 10 300 tools/bin/w43_bench 32 10 > $O/w43_b1.log 2>&1; rc=$?
grep -h "^b1\|^e64\|block1\|total" $O/w43_b1.log
exit $rc
