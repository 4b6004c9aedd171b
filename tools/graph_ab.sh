cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
GC_GRAPH=50 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread -k "step_random" > gpurun_out/pt.log 2>&1 || { tail -20 gpurun_out/pt.log; exit 1; }
tail -1 gpurun_out/pt.log
for v in 0 10 50 100; do
  GC_GRAPH=$v timeout -k 10 120 python bench.py --perft-roots 0 --no-cpu-baseline --fused-plies 0 > gpurun_out/bg$v.log 2>&1 || exit 1
  python -c "
import json
d=json.loads(open('gpurun_out/bg$v.log').read().strip().splitlines()[-1]); print('graph $v', d['value'], d['ms_per_step']*1000, d['roofline']['avg_launch_us'])"
done
