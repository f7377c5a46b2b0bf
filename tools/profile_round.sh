#!/bin/bash
# GPU-box profiling sequence for one round: full bench (with CPU baseline),
# then for each arithmetic (winograd = the headline, exact, x3 = the opt-in leg):
# rocprofv3 kernel-trace stats -> FETCH_SIZE pass -> WRITE_SIZE pass
# (separate passes: FETCH_SIZE and WRITE_SIZE do not fit one TCC pass on
# gfx950) -> MFMA busy cycles + GRBM_GUI_ACTIVE pass (MFMA utilisation,
# effective clock).  Profiling passes run the headline only (--no-side) on one
# stream so per-kernel averages time un-overlapped launches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
step() {
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 3 "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping"; exit $rc; fi
}
[ -n "$NO_FULL" ] || step bench_full 600 python bench.py --steps 20 --warmup 3
# LEGS: extra profiled legs beside the precisions: config3 (Transformer),
# config4 (gammatone 32k frontend + forward) and window (predict.py windows:
# 192 x 5 s windows per call), headline arithmetic
for P in ${PRECISIONS:-winograd exact x3} ${LEGS}; do
  case $P in
    config3) A="--no-cpu-baseline --no-side --streams 1 --model transformer" ;;
    config4) A="--no-cpu-baseline --no-side --streams 1 --mode gamma" ;;
    window) A="--no-cpu-baseline --no-side --streams 1 --mode window" ;;
    *) A="--no-cpu-baseline --no-side --streams 1 --precision $P" ;;
  esac
  step kt_$P 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$P/kt -o kt -- python bench.py --steps 10 --warmup 2 $A
  step fetch_$P 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/$P/pmc_fetch -o pmc -- python bench.py --steps 3 --warmup 1 $A
  step write_$P 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/$P/pmc_write -o pmc -- python bench.py --steps 3 --warmup 1 $A
  step mfma_$P 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/$P/pmc_mfma -o pmc -- python bench.py --steps 3 --warmup 1 $A
done
echo ALLDONE
