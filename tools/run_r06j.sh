#!/bin/bash
# Round-6 session J: the rollout's two variants (k_env_rollout4<true>: the window's occupancy
# filter, <false>: the table probed every ply) chosen per launch by its plies
# (gc_env_rollout_occ_min_plies); parity of both, then a same-box sweep over K with the
# threshold forced to always (0) and never (100000)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_full_width_digest.py tests/test_full_size.py -x -v -m gpu \
  --timeout 600 --timeout-method thread > gpurun_out/r06j_pytest.log 2>&1 || { echo "PYTEST rc=$?"; tail -30 gpurun_out/r06j_pytest.log; exit 3; }
tail -4 gpurun_out/r06j_pytest.log
L=gym-chess_amd/gym_chess_amd/libgymchess.so
KS="20 40 64 100 300 1000" LIBS="$L@GC_OCC_MIN_PLIES=0 $L@GC_OCC_MIN_PLIES=100000" REPS=${REPS:-3} bash tools/ab.sh || exit 5
