# PC sampling of the step kernel (diagnostic): stochastic, cycle-based
cd ${GRAFT_REPO_ROOT:-.}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles --pc-sampling-interval 65536 -d gpurun_out/pcs -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 300 --warmup 400 --fused-plies 0 --perft-roots 0 > gpurun_out/pcs.log 2>&1
rc=$?
tail -5 gpurun_out/pcs.log
ls -la gpurun_out/pcs 2>/dev/null
exit $rc
