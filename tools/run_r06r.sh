#!/bin/bash
# Round-6 session R: the API step's workgroups taking turns by phase (in-tree, GC_API_FAIR=1)
# against the old priorities (apif0); parity first, then the API legs
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
L=gym-chess_amd/gym_chess_amd/libgymchess.so
timeout -k 10 600 python -u -m pytest tests/test_api_step.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r06r_pytest.log 2>&1 || { echo "PYTEST rc=$?"; tail -20 gpurun_out/r06r_pytest.log; exit 3; }
tail -2 gpurun_out/r06r_pytest.log
MODE=api PARITY=1 LIBS="$L tools/_lib_apif0.so" REPS=${REPS:-5} bash tools/ab.sh || exit 5
