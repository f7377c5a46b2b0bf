#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -DSEDX_GRU_STAMPS -o /tmp/gru_bench tools/gru_bench.cpp sound-event-detection_amd/csrc/gru.hip || exit 1
timeout -k 10 120 /tmp/gru_bench 32 125 | tee gpurun_out/gru_bench.log
