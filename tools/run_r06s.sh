#!/bin/bash
# Round-6 session S: the paired fused kernel's workgroups taking turns ply by ply (in-tree,
# GC_PAIR_FAIR=1) against the old form (pf0): parity of the paired paths, then the fused variants
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
L=gym-chess_amd/gym_chess_amd/libgymchess.so
timeout -k 10 900 python -u -m pytest tests/test_opponent_mode.py tests/test_fide.py tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r06s_pytest.log 2>&1 || { echo "PYTEST rc=$?"; tail -20 gpurun_out/r06s_pytest.log; exit 3; }
tail -2 gpurun_out/r06s_pytest.log
MODE=var PARITY=1 LIBS="$L tools/_lib_pf0.so" REPS=${REPS:-3} bash tools/ab.sh || exit 5
