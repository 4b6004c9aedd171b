cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_single_env.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pt_single.log 2>&1 || { tail -40 gpurun_out/pt_single.log; exit 1; }
tail -3 gpurun_out/pt_single.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --variant-steps 0 --api-steps 0 --launched-steps 0 > gpurun_out/b_single.log 2>&1 || { tail -20 gpurun_out/b_single.log; exit 1; }
python -c "
import json;d=json.loads(open('gpurun_out/b_single.log').read().strip().splitlines()[-1]);print(json.dumps(d['single_env'])); p=d['perft']; print(p['value']/1e12, p['roofline']['kernel_ms'], p.get('oracle_checked_roots'))"
STEPS="pytest" bash tools/gpu_run.sh
