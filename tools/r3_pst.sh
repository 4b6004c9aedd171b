cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 120 python tools/pstamp_probe.py 65536 200 > gpurun_out/pst.log 2>&1; cat gpurun_out/pst.log
