#!/bin/bash
# Diagnostic: bench main leg for the in-tree library and each tools/_lib_<tag>.so given
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
B="--perft-roots 0 --no-cpu-baseline --variant-steps 0 --api-steps 0 --single-episodes 0"
timeout -k 10 120 python bench.py $B > gpurun_out/ab_base.log 2>&1 || { tail -5 gpurun_out/ab_base.log; exit 1; }
python tools/ab_show.py base gpurun_out/ab_base.log
for t in "$@"; do
  timeout -k 10 120 python tools/ab_parity.py tools/_lib_$t.so > gpurun_out/abp_$t.log 2>&1 || { echo "PARITY FAILED $t"; tail -5 gpurun_out/abp_$t.log; exit 1; }
  timeout -k 10 120 python tools/ab_lib.py tools/_lib_$t.so $B > gpurun_out/ab_$t.log 2>&1 || { tail -5 gpurun_out/ab_$t.log; exit 1; }
  python tools/ab_show.py $t gpurun_out/ab_$t.log
done
timeout -k 10 120 python bench.py $B > gpurun_out/ab_base2.log 2>&1 || exit 1
python tools/ab_show.py base2 gpurun_out/ab_base2.log
