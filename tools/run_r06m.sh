#!/bin/bash
# Round-6 session M: where the occupancy filter computes the post-move board's key -- Q1 in
# phase 1 (the in-tree build), Q0 in phase 0 (k1), Q3 in phase 1 with Q1's lookup in phase 2
# (k2) -- with the filter forced on, parity first
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
L=gym-chess_amd/gym_chess_amd/libgymchess.so
KS="300 1000" PARITY=1 LIBS="$L@GC_OCC_MIN_PLIES=0 tools/_lib_k1.so@GC_OCC_MIN_PLIES=0 tools/_lib_k2.so@GC_OCC_MIN_PLIES=0" REPS=${REPS:-3} bash tools/ab.sh || exit 5
