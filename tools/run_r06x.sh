#!/bin/bash
# Round-6 session X: the paired fused kernel's turns of 1 ply (in-tree) or 4 plies (pts2)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
L=gym-chess_amd/gym_chess_amd/libgymchess.so
MODE=var PARITY=1 LIBS="$L tools/_lib_pts2.so" REPS=${REPS:-4} bash tools/ab.sh || exit 5
