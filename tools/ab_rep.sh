#!/bin/bash
# Diagnostic: alternate bench main-leg runs of several library builds, R rounds
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
B="--perft-roots 0 --no-cpu-baseline --variant-steps 0 --api-steps 0 --single-episodes 0 ${BENCH_EXTRA:-}"
for r in $(seq ${R:-3}); do
  for t in "$@"; do
    timeout -k 10 120 python tools/ab_lib.py tools/_lib_$t.so $B > gpurun_out/ab_$t.log 2>&1 || { tail -5 gpurun_out/ab_$t.log; exit 1; }
    python -c "
import json
d=json.loads([l for l in open('gpurun_out/ab_$t.log').read().splitlines() if l.startswith('{')][-1])
print('$t', round(d['value']/1e9,3), round(d['roofline']['avg_launch_us'],2), 'us; launched', round(d.get('launched_step',{}).get('value',0)/1e9,3))"
  done
done
