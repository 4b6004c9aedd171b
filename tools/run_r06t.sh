#!/bin/bash
# Round-6 session T: the rollout's workgroups taking turns by ply (in-tree) or by the wall clock
# in periods of 1.28 / 2.56 / 5.12 us (f2s7 / f2s8 / f2s9); parity first
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
L=gym-chess_amd/gym_chess_amd/libgymchess.so
PARITY=1 LIBS="$L tools/_lib_f2s7.so tools/_lib_f2s8.so tools/_lib_f2s9.so" REPS=${REPS:-3} bash tools/ab.sh || exit 5
