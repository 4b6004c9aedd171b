#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
L="tools/_lib_role.so gym-chess_amd/gym_chess_amd/libgymchess.so"
PYTEST=1 REPS=2 LIBS="$L" bash tools/r3_ab.sh || exit $?
LIBS="$L" bash tools/r3_perft_ab.sh || exit $?
STEPS="pmcrf pmcrw pmcrm pmcpf pmcpw pmcpm" PROFILE_TAG=r03_v5 bash tools/gpu_run.sh
