cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_single_env.py tests/test_gpu_parity.py -x -q -m gpu -k "single or perft" --timeout 300 --timeout-method thread > gpurun_out/pt_q.log 2>&1 || { tail -40 gpurun_out/pt_q.log; exit 1; }
tail -2 gpurun_out/pt_q.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --variant-steps 0 --api-steps 0 --launched-steps 0 --no-cpu-baseline > gpurun_out/b_q.log 2>&1 || { tail -20 gpurun_out/b_q.log; exit 1; }
python -c "
import json;d=json.loads(open('gpurun_out/b_q.log').read().strip().splitlines()[-1]);s=d['single_env'];print('single', s['value'], s['engine_get_possible_moves']['value']); p=d['perft']; print('perft', p['value']/1e12, p['roofline']['kernel_ms'], p.get('oracle_checked_roots'), p.get('oracle_subsample'))"
