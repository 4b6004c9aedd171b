#!/bin/bash
# same-box A/B: two quads per workgroup (this build) vs four (QUADS_WG=4: one workgroup per CU)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
M=gym-chess_amd/gym_chess_amd/libgymchess.so
REPS=3 LIBS="$M tools/_lib_qw4.so" bash tools/r3_ab.sh
