#!/bin/bash
# same-box A/B: the role pairing of a workgroup's two quads (GC_QXOR 2 = HEAD, 1, 3) and one quad
# per workgroup (QUADS_WG=1)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
M=gym-chess_amd/gym_chess_amd/libgymchess.so
REPS=2 LIBS="$M tools/_lib_qx1.so tools/_lib_qx3.so tools/_lib_qw1.so" bash tools/r3_ab.sh
