#!/bin/bash
# Block 1 with conv1 inside the Winograd launch: its parity tests, then the
# headline A/B of --wino-block1 1 (separate conv1 launch) / 2 (fused) and of
# the fused kernel's weight-load variant (build/ab/pre), alternating rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread \
  -k "${PYTEST_K:-block1 or stage_goldens}" > gpurun_out/t2.log 2>&1; rc=$?
tail -25 gpurun_out/t2.log
[ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for v in tree:1 tree:2 ${VARIANTS:-pre:2}; do
    pkg=${v%%:*}; wb=${v##*:}
    if [ $pkg = tree ]; then P=""; else P="--ab-package $PWD/sound-event-detection_amd/build/ab/$pkg"; fi
    timeout -k 10 200 python bench.py $P --steps 20 --warmup 3 --no-side --no-cpu-baseline --wino-block1 $wb \
      > gpurun_out/ab_${pkg}_$wb$r.log 2>&1 || exit $?
    python3 -c "
import json
s=open('gpurun_out/ab_${pkg}_$wb$r.log').read(); d=json.loads(s[s.rfind('{\"metric\"'):].split('\n')[0])
st=d['stage_ms']; iso=d.get('stage_ms_isolated') or {}
print('$pkg wb=$wb round $r', d['value'], 'clips/s', d['ms_per_step'], 'ms/step | timed b1c1 %s b1c2 %s | iso b1c1 %s b1c2 %s' % (st.get('b1c1'), st.get('b1c2'), iso.get('b1c1'), iso.get('b1c2')))"
  done
done
