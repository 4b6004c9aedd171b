#!/bin/bash
# Round-6 session O: which of a CU's two workgroups runs the slow plies (index, start, SIMDs)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
for k in 1000; do
  PST_QUAD=1 PST_LIB=tools/_lib_pst.so timeout -k 10 120 python tools/pstamp_probe.py 65536 $k > gpurun_out/r06o_pst_$k.log 2>&1 || { echo "pst $k rc=$?"; tail -5 gpurun_out/r06o_pst_$k.log; exit 3; }
  head -1 gpurun_out/r06o_pst_$k.log; tail -14 gpurun_out/r06o_pst_$k.log
done
