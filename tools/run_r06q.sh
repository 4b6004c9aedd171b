#!/bin/bash
# Round-6 session Q: the filter's crossover again, with the workgroups taking turns (GC_WG_FAIR=1)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
L=gym-chess_amd/gym_chess_amd/libgymchess.so
KS="20 100 300 500 700 1000 2000" LIBS="$L@GC_OCC_MIN_PLIES=0 $L@GC_OCC_MIN_PLIES=100000" REPS=${REPS:-3} bash tools/ab.sh || exit 5
