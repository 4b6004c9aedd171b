cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 120 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "rollout_device_trace or step_random_per_ply" --timeout 120 --timeout-method thread > gpurun_out/pt_sp.log 2>&1 || { tail -20 gpurun_out/pt_sp.log; exit 1; }
echo "in-tree (split 0) parity ok"
PST_LIB=tools/_lib_pst2.so timeout -k 10 120 python tools/pstamp_probe.py 65536 200 > gpurun_out/pst2.log 2>&1; cat gpurun_out/pst2.log
bash tools/ab_libs.sh sp1 sp2 && bash tools/ab_libs.sh sp2 sp1
