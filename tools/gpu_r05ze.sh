#!/bin/bash
# Round 5: batches in flight A/B (bench --streams 2 vs 3), headline leg only
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05ze
mkdir -p $O
for r in 1 2; do
  for s in 2 3; do
    timeout -k 10 300 python -u bench.py --streams $s --steps 20 --warmup 3 --no-cpu-baseline --no-side > $O/s${s}_$r.log 2>&1 || { tail -20 $O/s${s}_$r.log; exit 1; }
    echo "streams $s round $r: $(grep -o '"value": [0-9.]*' $O/s${s}_$r.log | head -1) $(grep -o '"ms_per_clip_p50": [0-9.]*' $O/s${s}_$r.log | head -1)"
  done
done | tee $O/ab.txt
