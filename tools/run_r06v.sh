#!/bin/bash
# Round-6 session V: the workgroups' turns of 1 ply (in-tree), 2 plies (ts1) and 4 plies (ts2)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
L=gym-chess_amd/gym_chess_amd/libgymchess.so
PARITY=1 LIBS="$L tools/_lib_ts1.so tools/_lib_ts2.so" REPS=${REPS:-3} bash tools/ab.sh || exit 5
