#!/bin/bash
# Round-6 session P: the two workgroups of a CU taking turns one priority level up, ply by ply
# (GC_WG_FAIR=1: fair), against the in-tree build; stamps of the fair build; parity first
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
PST_QUAD=1 PST_LIB=tools/_lib_pstfair.so timeout -k 10 120 python tools/pstamp_probe.py 65536 1000 > gpurun_out/r06p_pstfair_1000.log 2>&1 || { echo "pst rc=$?"; tail -5 gpurun_out/r06p_pstfair_1000.log; exit 3; }
head -1 gpurun_out/r06p_pstfair_1000.log; tail -9 gpurun_out/r06p_pstfair_1000.log
L=gym-chess_amd/gym_chess_amd/libgymchess.so
KS="20 300 1000" PARITY=1 LIBS="$L tools/_lib_fair.so" REPS=${REPS:-3} bash tools/ab.sh || exit 5
