cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
for k in 20 1000; do timeout -k 10 120 python tools/pstamp_probe.py 65536 $k > gpurun_out/pst_$k.log 2>&1; cat gpurun_out/pst_$k.log; done
