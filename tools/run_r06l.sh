#!/bin/bash
# Round-6 session L: where the fused rollout's slow waves run (tools/pstamp_probe.py with the
# placement of every quad wave: by XCD, by CU, the two workgroups of a CU), the filter's variant
# at K = 1 000 and the plain one at K = 300
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
for k in 300 1000; do
  PST_QUAD=1 PST_LIB=tools/_lib_pst.so timeout -k 10 120 python tools/pstamp_probe.py 65536 $k > gpurun_out/r06l_pst_$k.log 2>&1 || { echo "pst $k rc=$?"; tail -5 gpurun_out/r06l_pst_$k.log; exit 3; }
  head -1 gpurun_out/r06l_pst_$k.log; tail -8 gpurun_out/r06l_pst_$k.log
done
