cd ${GRAFT_REPO_ROOT:-.}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1 || { tail -20 gpurun_out/pt.log; exit 1; }
tail -1 gpurun_out/pt.log
timeout -k 10 120 python bench.py --perft-roots 0 --no-cpu-baseline --fused-plies 0 > gpurun_out/b2.log 2>&1 || exit 1
python -c "
import json
d=json.loads(open('gpurun_out/b2.log').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['avg_launch_us'])"
timeout -k 10 60 python tools/stamp_probe2.py
