#!/bin/bash
# GPU-box profiling sequence: full bench (with CPU baseline) -> rocprofv3
# kernel-trace stats -> FETCH_SIZE pass -> WRITE_SIZE pass (separate passes:
# FETCH_SIZE and WRITE_SIZE do not fit one TCC pass on gfx950) -> MFMA busy
# cycles + GRBM_GUI_ACTIVE pass (MFMA utilisation, effective clock).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
TAG=${TAG:-r01}
ARGS="${BENCH_ARGS:-}"
step() {
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 5 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping"; exit $rc; fi
}
step bench_full 600 python bench.py --steps 20 --warmup 3 $ARGS
step kt 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-side --streams 1 $ARGS
step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o pmc -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-side --streams 1 $ARGS
step pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o pmc -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-side --streams 1 $ARGS
step pmc_mfma 600 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_mfma -o pmc -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-side --streams 1 $ARGS
echo ALLDONE
