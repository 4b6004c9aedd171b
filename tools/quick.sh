# quick A/B: parity subset, bench (paired vs one-wave kernel), stamps of the paired kernel
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1 || { tail -20 gpurun_out/pt.log; exit 1; }
tail -1 gpurun_out/pt.log
for v in "pair:X=1" "one:GC_STEP1=1" "pair2:X=2"; do
  n=${v%%:*}; ev=${v#*:}
  env $ev timeout -k 10 120 python bench.py --perft-roots 0 --no-cpu-baseline > gpurun_out/b_$n.log 2>&1 || exit 1
  python -c "
import json
d=json.loads(open('gpurun_out/b_$n.log').read().strip().splitlines()[-1]); print('$n', round(d['value']/1e9,3), 'e9', round(d['roofline']['avg_launch_us'],2), 'us; fused', round(d['fused_rollout']['value']/1e9,3), 'e9', round(d['fused_rollout']['kernel_ms']*1000/200,2), 'us/ply')"
done
[ -f tools/_build_stamps.so ] && timeout -k 10 60 python tools/stamp_probe2.py
