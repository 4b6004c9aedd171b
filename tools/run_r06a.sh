#!/bin/bash
# Round-6 session A: the full-width digests (headline kernel with Q1's late commit, and the
# random opponent for both colours) and the full-size tests, then a same-box A/B of the late
# commit against the phase-2 commit (tools/_lib_late0.so), then the phase stamps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_full_width_digest.py tests/test_full_size.py -x -v -m gpu \
  --timeout 600 --timeout-method thread > gpurun_out/r06a_pytest.log 2>&1 || { echo "PYTEST rc=$?"; tail -30 gpurun_out/r06a_pytest.log; exit 3; }
tail -8 gpurun_out/r06a_pytest.log
LIBS="tools/_lib_late0.so tools/_lib_ring0.so gym-chess_amd/gym_chess_amd/libgymchess.so" REPS=${REPS:-3} bash tools/ab.sh || exit 4
STEPS="pst" bash tools/gpu_run.sh || exit 5
