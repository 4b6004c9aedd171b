cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
STEPS="smoke pytest short" PROFILE_TAG=r03_v3 bash tools/gpu_run.sh
