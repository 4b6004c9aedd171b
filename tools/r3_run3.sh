cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_spill.py tests/test_checkpoint.py tests/test_opponent_mode.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pt_spill.log 2>&1 || { tail -30 gpurun_out/pt_spill.log; exit 1; }
tail -3 gpurun_out/pt_spill.log
STEPS="pytest" bash tools/gpu_run.sh
