#!/bin/bash
# Round 5: gamma_erb with 3 register stages (build/abx/erb3, -DSEDX_ERB_STAGES=3) against
# (historical: the 3-stage variant was measured slower and removed; this script no longer runs as is)
# the tree's 2: config-4 frontend time, alternating rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05zf
mkdir -p $O
for r in 1 2 3; do
  for v in tree erb3; do
    if [ $v = tree ]; then P=""; else P="--ab-package $PWD/sound-event-detection_amd/build/abx/$v"; fi
    timeout -k 10 300 python -u bench.py $P --mode gamma --steps 5 --warmup 2 --no-cpu-baseline --no-side > $O/ab_${v}_$r.log 2>&1 || { tail -20 $O/ab_${v}_$r.log; exit 1; }
    echo "$v round $r: $(grep -o '"gamma_frontend": {"ms_per_batch": [0-9.]*' $O/ab_${v}_$r.log | head -1) $(grep -o '"value": [0-9.]*' $O/ab_${v}_$r.log | head -1)"
  done
done | tee $O/ab.txt
