#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
M=gym-chess_amd/gym_chess_amd/libgymchess.so
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 3; }
tail -1 gpurun_out/smoke.log
GC_NO_QUAD=1 timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_pair.log 2>&1; echo "pytest pair-early rc=$?"; tail -2 gpurun_out/pytest_pair.log
REPS=2 LIBS="$M@GC_NO_QUAD=1 tools/_lib_quad.so@GC_NO_QUAD=1 tools/_lib_noprobe.so@GC_NO_QUAD=1 $M" bash tools/r3_ab.sh
