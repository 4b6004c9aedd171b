#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
B="--no-cpu-baseline --launched-steps 0 --api-steps 0 --single-episodes 0 --variant-steps 0 --perft-roots 0"
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 $B > gpurun_out/bs$r.log 2>&1 || { tail -5 gpurun_out/bs$r.log; exit 3; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/bs$r.log') if l.startswith('{')][-1]); print('bench K=20', round(d['value']/1e9,3), 'wall us', round(d['timed_region_ms']*1e3,1), 'event us', round(d['event_ms_per_step']*20e3,1))"
done
timeout -k 10 200 python bench.py --steps 1000 --warmup 5 $B > gpurun_out/bl.log 2>&1 || { tail -5 gpurun_out/bl.log; exit 3; }
python -c "import json; d=json.loads([l for l in open('gpurun_out/bl.log') if l.startswith('{')][-1]); print('bench K=1000', round(d['value']/1e9,3), 'wall us', round(d['timed_region_ms']*1e3,1), 'event us', round(d['event_ms_per_step']*1000e3,1))"
