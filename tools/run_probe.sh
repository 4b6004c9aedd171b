#!/bin/bash
# one diagnostic gpurun session: the launch / region anatomy probes (each under its own limit)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 120 tools/_region_anatomy > gpurun_out/anatomy.jsonl 2>&1 || { tail -5 gpurun_out/anatomy.jsonl; exit 3; }
for k in 20 1000; do PST_QUAD=1 PST_LIB=tools/_lib_pst.so timeout -k 10 120 python tools/pstamp_probe.py 65536 $k > gpurun_out/pst_$k.log 2>&1 || exit 3; done
cat gpurun_out/anatomy.jsonl; head -3 gpurun_out/pst_20.log
