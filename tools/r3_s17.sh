#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
M=gym-chess_amd/gym_chess_amd/libgymchess.so
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 3; }
tail -1 gpurun_out/smoke.log
PYTEST=1 REPS=2 LIBS="tools/_lib_q7.so $M" bash tools/r3_ab.sh
PST_QUAD=1 PST_LIB=tools/_lib_pstq.so timeout -k 10 120 python tools/pstamp_probe.py 65536 1000 > gpurun_out/pstq.log 2>&1; tail -32 gpurun_out/pstq.log
