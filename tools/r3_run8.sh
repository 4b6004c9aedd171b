cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_api_step.py tests/test_spill.py -x -q -m gpu -k "random_opponent or growth" --timeout 300 --timeout-method thread > gpurun_out/pt_new.log 2>&1 || { tail -40 gpurun_out/pt_new.log; exit 1; }
tail -2 gpurun_out/pt_new.log
STEPS="smoke pytest short" PROFILE_TAG=r03_v3 bash tools/gpu_run.sh
