#!/bin/bash
# perft split pass in move-count order (k_expand_count / k_expand_place / k_perft2_rec): parity,
# A/B against the gathering form, and the leaf kernel's PMC traffic
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "perft or smoke or fide" --timeout 300 --timeout-method thread > gpurun_out/pytest_perft.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_perft.log; [ $rc -le 1 ] || exit 3
M=gym-chess_amd/gym_chess_amd/libgymchess.so
REPS=2 LIBS="$M@GC_PERFT_GATHER=1 $M" bash tools/r3_perft_ab.sh || exit 3
STEPS="pmcpf pmcpw pmcpm" PROFILE_TAG=r03_v7 bash tools/gpu_run.sh
