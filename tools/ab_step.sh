#!/bin/bash
# A/B of step_random variants on one box: parity subset, then the bench's main leg under
# each variant (env assignments per run, e.g. GC_STREAMS=2).
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
GC_STREAMS=${PARITY_STREAMS:-2} timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "step_random or rollout or weird" --timeout 120 --timeout-method thread > gpurun_out/ab_pt.log 2>&1 || { tail -30 gpurun_out/ab_pt.log; exit 1; }
tail -1 gpurun_out/ab_pt.log
B="python bench.py --perft-roots 0 --no-cpu-baseline --variant-steps 0 --api-steps 0 --single-episodes 0"
for v in ${VARIANTS:-"s1:GC_STREAMS=1" "s2:GC_STREAMS=2" "s4:GC_STREAMS=4"}; do
  n=${v%%:*}; ev=${v#*:}; ev=${ev//+/ }
  env $ev timeout -k 10 120 $B > gpurun_out/ab_$n.log 2>&1 || { tail -5 gpurun_out/ab_$n.log; exit 1; }
  python -c "
import json
d=json.loads(open('gpurun_out/ab_$n.log').read().strip().splitlines()[-1]); print('$n', round(d['value']/1e9,3), 'e9', round(d['roofline']['avg_launch_us'],2), 'us; launched', round(d.get('launched_step',{}).get('value',0)/1e9,3), 'e9')"
done
