#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
PYTEST=1 REPS=2 LIBS="tools/_lib_nofair.so tools/_lib_rolert.so gym-chess_amd/gym_chess_amd/libgymchess.so" bash tools/r3_ab.sh || exit $?
sed -i 's/^STEPS="pmcpf pmcpw".*$//' tools/r3_s5.sh
bash tools/r3_s5.sh || exit $?
STEPS="pmcpf pmcpw" PROFILE_TAG=r03_v5 bash tools/gpu_run.sh
