# A/B of the step kernels: parity subset for each variant, then bench lines + stamps
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread -k "step_random or rollout or env" > gpurun_out/pt.log 2>&1 || { tail -20 gpurun_out/pt.log; exit 1; }
GC_SPLIT=1 $T 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread -k "step_random" > gpurun_out/pt_split.log 2>&1 || { tail -20 gpurun_out/pt_split.log; exit 1; }
tail -1 gpurun_out/pt.log gpurun_out/pt_split.log
for v in "b1:GC_STEP1=1" "b2:X=1" "b3:GC_SPLIT=1"; do
  n=${v%%:*}; ev=${v#*:}
  env $ev $T 120 python bench.py --perft-roots 0 --no-cpu-baseline --fused-plies 0 > gpurun_out/$n.log 2>&1 || exit 1
done
python -c "
import json
for f in ('b1','b2','b3'):
    d=json.loads(open('gpurun_out/'+f+'.log').read().strip().splitlines()[-1]); print(f, d['value'], d['roofline']['avg_launch_us'])"
if [ -f tools/_build_stamps.so ]; then
  $T 60 python tools/stamp_probe2.py > gpurun_out/st_b2.log 2>&1 || exit 1
  GC_SPLIT=1 $T 60 python tools/stamp_probe2.py > gpurun_out/st_b3.log 2>&1 || exit 1
  cat gpurun_out/st_b2.log gpurun_out/st_b3.log
fi
