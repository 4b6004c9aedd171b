#!/bin/bash
# Round-6 session I: the in-tree build (occupancy filter v3 + the next draw's Philox word in
# phase 3) at full width against the oracle, then a same-box A/B of the placements
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_full_width_digest.py tests/test_full_size.py tests/test_long_horizon.py -x -v -m gpu \
  -k "digest or full_size or 777001" --timeout 600 --timeout-method thread > gpurun_out/r06i_pytest.log 2>&1 || { echo "PYTEST rc=$?"; tail -30 gpurun_out/r06i_pytest.log; exit 3; }
tail -4 gpurun_out/r06i_pytest.log
PARITY=1 LIBS="tools/_lib_occ0.so gym-chess_amd/gym_chess_amd/libgymchess.so tools/_lib_p2.so tools/_lib_nophx.so tools/_lib_occ0phx.so tools/_lib_wg1.so tools/_lib_p2wg1.so" REPS=${REPS:-5} bash tools/ab.sh || exit 5
