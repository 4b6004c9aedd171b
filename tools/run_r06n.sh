#!/bin/bash
# Round-6 session N: the filter's fast lanes read one shared line (the init block: every wave of
# an XCD on one L2 channel) or slot 0 of their own table (fs1: 64 contiguous lines per wave, hot
# in L2); the filter forced on, and off for reference; parity first
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
L=gym-chess_amd/gym_chess_amd/libgymchess.so
KS="20 300 1000" PARITY=1 LIBS="$L@GC_OCC_MIN_PLIES=0 tools/_lib_fs1.so@GC_OCC_MIN_PLIES=0 $L@GC_OCC_MIN_PLIES=100000" REPS=${REPS:-3} bash tools/ab.sh || exit 5
