cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
GC_SPIN_US=0 timeout -k 10 180 python tools/short_probe.py --streams 1,2 --reps 3 > gpurun_out/sp_block.log 2>&1 || exit 1
timeout -k 10 180 python tools/short_probe.py --streams 1,2 --reps 3 > gpurun_out/sp_spin.log 2>&1 || exit 1
GC_SPIN_US=0 timeout -k 10 180 python tools/short_probe.py --fused --streams 1 --reps 4 > gpurun_out/sp_fblock.log 2>&1 || exit 1
timeout -k 10 180 python tools/short_probe.py --fused --streams 1 --reps 4 > gpurun_out/sp_fspin.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread -k "rollout or step_random" > gpurun_out/pt_roll.log 2>&1 || exit 1
echo done
