#!/bin/bash
# Round-6 session W: the workgroups' turns at K = 20 only, 8 interleaved repeats: 1 ply (in-tree),
# 4 plies (ts2), 8 plies (ts3)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
L=gym-chess_amd/gym_chess_amd/libgymchess.so
KS="20" LIBS="$L tools/_lib_ts2.so tools/_lib_ts3.so" REPS=${REPS:-8} bash tools/ab.sh || exit 5
