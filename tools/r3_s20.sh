#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
PST_QUAD=1 PST_LIB=tools/_lib_pstq.so timeout -k 10 120 python tools/pstamp_probe.py 65536 1000 > gpurun_out/pstq.log 2>&1; tail -40 gpurun_out/pstq.log
