#!/bin/bash
# Diagnostic: the bench's perft leg for the in-tree library and each tools/_lib_<tag>.so given
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
B="--steps 5 --warmup 5 --settle 0 --launched-steps 0 --variant-steps 0 --api-steps 0 --single-episodes 0 --no-cpu-baseline --oracle-perft-roots 0"
show() { python -c "
import json
d=json.loads([l for l in open('$2') if l.startswith('{')][-1]); p=d['perft']
print('$1', round(p['value']/1e12,4), 'e12 nodes/s', round(p['roofline']['kernel_ms'],1), 'ms leaf')"; }
timeout -k 10 120 python bench.py $B > gpurun_out/abp_base.log 2>&1 || { tail -5 gpurun_out/abp_base.log; exit 1; }
show base gpurun_out/abp_base.log
for t in "$@"; do
  timeout -k 10 120 python tools/ab_lib.py tools/_lib_$t.so $B > gpurun_out/abp_$t.log 2>&1 || { tail -5 gpurun_out/abp_$t.log; exit 1; }
  show $t gpurun_out/abp_$t.log
done
