cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 120 python tools/short_probe.py --fused --streams 1 --reps 3 --ks 5,10,20,40,100,1000 > gpurun_out/sp_fk.log 2>&1 || exit 1
STEPS="short calib pmcrf pmcrw pmcrm" PROFILE_TAG=r03_v1 bash tools/gpu_run.sh
