#!/bin/bash
# A/B of two builds of the package on one GPU box (box-to-box variance is
# 3-5 %, so variants are only compared inside one call):
#   VARIANTS="name=pkgdir ..." ROUNDS=3 bash tools/ab_bench.sh
# Runs the bench alternately (A B A B ...) and prints value + conv stage times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
ROUNDS=${ROUNDS:-3}
for r in $(seq 1 "$ROUNDS"); do
  for v in $VARIANTS; do
    name=${v%%=*}; pkg=${v#*=}
    SEDX_PKG=$pkg timeout -k 10 180 python bench.py --steps ${STEPS:-30} --warmup 5 --no-cpu-baseline --no-exact \
      ${BENCH_ARGS} > gpurun_out/ab/$name.$r.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "== $name round $r rc=$rc"; tail -20 gpurun_out/ab/$name.$r.log; exit $rc; fi
    python - "$name" "$r" gpurun_out/ab/$name.$r.log <<'EOF'
import json, sys
line = [l for l in open(sys.argv[3]) if l.startswith('{')][-1]
d = json.loads(line)
st = d.get('stage_ms') or {}
print('%-8s r%s value %8.1f  ' % (sys.argv[1], sys.argv[2], d['value']) +
      ' '.join('%s=%.4f' % (k, v) for k, v in st.items() if isinstance(v, (int, float))), flush=True)
EOF
  done
done
