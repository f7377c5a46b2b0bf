#!/bin/bash
# GRU recurrence micro-benchmark.  BUILD=1 (here): tools/bin/gru_bench with
# per-phase s_memtime stamps; RUN=1 (GPU box): B in $BATCHES (default 1 32).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out tools/bin
if [ -n "$BUILD" ]; then
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fno-slp-vectorize -fno-vectorize -Wno-unused-result \
    -DSEDX_GRU_STAMPS -Isound-event-detection_amd/csrc -o tools/bin/gru_bench tools/gru_bench.cpp \
    sound-event-detection_amd/csrc/gru.hip || exit 1
fi
[ -n "$RUN" ] || exit 0
for b in ${BATCHES:-1 32}; do
  timeout -k 10 120 tools/bin/gru_bench $b 125 | tee -a gpurun_out/gru_bench.log || exit $?
done
