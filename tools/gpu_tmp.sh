cd $GRAFT_REPO_ROOT
RUN=1 VARIANTS="full nb4 i3" BATCHES=32 REPS=30 bash tools/gpu_wino.sh 2>&1 | grep -E "==|total" || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "wino" > gpurun_out/t_wino.log 2>&1; rc=$?; grep -E "passed|failed" gpurun_out/t_wino.log | tail -2; exit $rc
