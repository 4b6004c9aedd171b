cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
STEPS="pytest short calib" PROFILE_TAG=r03_v0 bash tools/gpu_run.sh
