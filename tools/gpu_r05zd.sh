#!/bin/bash
# Round 5: gamma spectrum with twiddles / window read per stage (SEDX_TUNE_GAMMA_SPEC 2 = 4 waves/SIMD,
# 3 = 5 waves/SIMD): gamma parity tests, then frontend A/B and a kernel trace
# (historical: variants 2 / 3 were measured slower and removed; this script no longer runs as is)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05zd
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "gamma" --timeout 200 --timeout-method thread > $O/pytest_gamma.log 2>&1 || { tail -30 $O/pytest_gamma.log; exit 1; }
tail -1 $O/pytest_gamma.log
for r in 1 2; do
  for v in 0 2 3; do
    timeout -k 10 300 python -u bench.py --mode gamma --gamma-spec $v --steps 5 --warmup 2 --no-cpu-baseline --no-side > $O/ab_${v}_$r.log 2>&1 || { tail -20 $O/ab_${v}_$r.log; exit 1; }
    echo "spec $v round $r: $(grep -o '"gamma_frontend": {"ms_per_batch": [0-9.]*' $O/ab_${v}_$r.log | head -1)"
  done
done | tee $O/ab.txt
cd /tmp && export TMPDIR=/tmp
for v in 0 3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_$v -o run -- python3 $GRAFT_REPO_ROOT/bench.py --mode gamma --gamma-spec $v --steps 3 --warmup 1 --no-cpu-baseline --no-side > $GRAFT_REPO_ROOT/$O/prof_$v.log 2>&1 || exit 1
done
find $GRAFT_REPO_ROOT/$O -name "*kernel_stats.csv" | head
