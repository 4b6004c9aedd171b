#!/bin/bash
# Round-6 session U: with the workgroups' turns, Q2 raised over Q0 from phase 1 (q2up1) or phase 2
# (q2up2) instead of phase 3 (in-tree); parity first
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
L=gym-chess_amd/gym_chess_amd/libgymchess.so
PARITY=1 LIBS="$L tools/_lib_q2up1.so tools/_lib_q2up2.so" REPS=${REPS:-3} bash tools/ab.sh || exit 5
