cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
STEPS="${STEPS:-smoke bench short prof profs calib pmcrf pmcrw pmcrm pmcpf pmcpw pmcpm pmcf pmcw pmcm}" PROFILE_TAG=${TAG:-r03_v2} bash tools/gpu_run.sh
