#!/bin/bash
# Round-6 session H: the launch anatomy at K = 20 (the driver's shape) and K = 1000, with and
# without the occupancy filter
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in pstocc0 pst; do
  for k in 20 1000; do
    PST_QUAD=1 PST_LIB=tools/_lib_$v.so timeout -k 10 120 python tools/pstamp_probe.py 65536 $k > gpurun_out/r06h_${v}_$k.log 2>&1 || { echo "PST $v rc=$?"; exit 3; }
    echo "== $v K=$k"; cat gpurun_out/r06h_${v}_$k.log
  done
done
