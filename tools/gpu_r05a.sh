#!/bin/bash
# Round 5, F(4x4,3x3): LDS-DMA out-of-range probe, the standalone F(4,3) vs
# F(2,3) vs float64 check + timing, ablation timings (halo DMA / U DMA /
# epilogue), then the winograd GPU tests and a short headline bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05a
mkdir -p $O
timeout -k 10 60 tools/bin/oob_lds_probe > $O/oob.log 2>&1 || exit 3
timeout -k 10 150 tools/bin/w43_bench 32 10 > $O/w43.log 2>&1; rc=$?
echo "w43 rc=$rc"; tail -n 4 $O/w43.log
[ $rc -eq 0 ] || exit 4
for v in abl1 abl2 abl4; do
  timeout -k 10 150 tools/bin/w43_bench_$v 32 10 > $O/w43_$v.log 2>&1; rc=$?
  [ $rc -le 1 ] || exit $rc
done
grep -h total $O/w43_abl*.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -k "wino and not x3" > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -n 3 $O/tests.log
[ $rc -eq 0 ] || exit 5
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-side > $O/bench.log 2>&1
