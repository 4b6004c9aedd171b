#!/bin/bash
# round-4 session: single-board env parity + probe, API-step priority A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp; mkdir -p gpurun_out
PYTEST_ARGS="tests/test_single_env.py tests/test_gpu_parity.py tests/test_lib_rs_quirks.py tests/test_opponent_mode.py tests/test_api_step.py" STEPS="pytest" bash tools/gpu_run.sh || exit $?
timeout -k 10 300 python tools/single_probe.py > gpurun_out/single_probe.json 2>&1 || exit 3
M=gym-chess_amd/gym_chess_amd/libgymchess.so
MODE=api REPS=2 LIBS="$M tools/_lib_ap1.so tools/_lib_ap2.so" bash tools/ab.sh
