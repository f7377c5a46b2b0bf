#!/bin/bash
# One gpurun call made of named steps (replaces round 5's per-call one-off
# scripts):  tools/gpu_session.sh TAG STEP [STEP ...]
# Outputs go under gpurun_out/TAG/<step>.log.  Every step runs under its own
# time limit; the session stops at the first step that fails, faults, aborts
# or times out (no retries).
#   smoke          __graft_entry__ build() + smoke()
#   tests          pytest -m gpu (all GPU tests)
#   tests=EXPR     pytest -m gpu -k EXPR  (',' in EXPR reads as ' ')
#   testsp=EXPR    the same with -s (the tests' printed errors in the log)
#   bench          python bench.py (default command)
#   bench=ARGS     python bench.py ARGS   (',' in ARGS reads as ' ')
#   w43=B          tools/run/w43_bench B 20 (build first: tools/build_w43.sh)
#   w43v=NAME:B    tools/run/w43_bench_NAME B 20 (a VARIANTS build)
#   w43o=ORDER:B   tools/run/w43_bench B 20 with W43_ORDER=ORDER (item order A/B)
#   w43s=B         tools/run/w43_bench B 20 with W43_SCHED=0 (static item order, no claims)
#   prof           tools/profile_round.sh (rocprof kernel trace + PMC passes; env as there)
#   ab=SETS        tools/ab_headline.sh: headline-leg A/B of '|'-separated bench argument sets (',' = ' ')
#   rank2          python bench.py --gpus 2 --backend gloo (the N > 1 path, both ranks on GPU 0)
#   sq             three rocprofv3 --pmc SQ passes of the headline (one stream) into gpurun_out/TAG/sq{1,2,3}
#                  (tools/sq_summary.py input)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:?tag}; shift
O=gpurun_out/$TAG
mkdir -p "$O"
n=0
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  n=$((n + 1))
  echo "== [$n] $name: $*"
  timeout -k 10 "$t" "$@" > "$O/$n.$name.log" 2>&1
  local rc=$?
  echo "== [$n] $name rc=$rc"; tail -n ${TAIL:-12} "$O/$n.$name.log" | cut -c1-400
  # (w43_bench exits 1 on a numerical MISMATCH — expected of ablation builds — and keeps going)
  if [ $rc -eq 1 ] && [[ $name == w43* ]]; then return 0; fi
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
for s in "$@"; do
  arg=${s#*=}; arg=${arg//,/ }
  case $s in
    smoke) step smoke 300 python -u -c "import __graft_entry__ as g; g.build(); g.smoke()" ;;
    tests) step pytest 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ;;
    testsp=*) step pytest 1100 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -k "$arg" ;;
    tests=*) step pytest 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$arg" ;;
    bench) step bench 600 python -u bench.py ;;
    bench=*) step bench 600 python -u bench.py $arg ;;
    w43=*) step w43_b$arg 200 tools/run/w43_bench $arg 20 ;;
    w43v=*) v=${arg%%:*}; b=${arg#*:}; step w43_${v}_b$b 200 tools/run/w43_bench_$v $b 20 ;;
    w43o=*) o=${arg%%:*}; b=${arg#*:}; step w43_o${o}_b$b 200 env W43_ORDER=$o tools/run/w43_bench $b 20 ;;
    w43s=*) step w43_static_b$arg 200 env W43_SCHED=0 tools/run/w43_bench $arg 20 ;;
    prof) step prof 1100 tools/profile_round.sh ;;
    ab=*) step ab 900 tools/ab_headline.sh "$TAG/ab$n" "${s#*=}" ${AB_ROUNDS:-2} ;;
    rank2) step rank2 600 python -u bench.py --gpus 2 --backend gloo ;;
    sq)
      A="--no-cpu-baseline --no-side --streams 1 --steps 3 --warmup 1"
      step sq1 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
        SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/sq1 -o p -- python bench.py $A
      step sq2 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT \
        SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU --output-format csv -d $O/sq2 -o p -- python bench.py $A
      step sq3 150 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM \
        SQ_ACTIVE_INST_SCA SQ_WAVES --output-format csv -d $O/sq3 -o p -- python bench.py $A ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "== session $TAG done"
