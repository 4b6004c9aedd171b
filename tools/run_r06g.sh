#!/bin/bash
# Round-6 session E: the occupancy filter v3 (in-tree build) at full width against the oracle;
# its phase stamps; parity gate and same-box A/B against the probe-every-ply build and the SIMD
# mappings; PMC traffic of the driver-shaped launch; the default bench line (new legs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_full_width_digest.py tests/test_full_size.py tests/test_long_horizon.py -x -v -m gpu \
  -k "digest or full_size or 777001" --timeout 600 --timeout-method thread > gpurun_out/r06g_pytest.log 2>&1 || { echo "PYTEST rc=$?"; tail -30 gpurun_out/r06g_pytest.log; exit 3; }
tail -8 gpurun_out/r06g_pytest.log
PST_QUAD=1 PST_WG=1 PST_LIB=tools/_lib_pstwg1.so timeout -k 10 120 python tools/pstamp_probe.py 65536 1000 > gpurun_out/r06g_pst.log 2>&1 || exit 4
cat gpurun_out/r06g_pst.log
PARITY=1 LIBS="tools/_lib_occ0.so gym-chess_amd/gym_chess_amd/libgymchess.so tools/_lib_wg1.so" REPS=${REPS:-5} bash tools/ab.sh || exit 5
PROFILE_TAG=r06_occ3q STEPS="pmcrf" bash tools/gpu_run.sh || exit 6
cat gpurun_out/summary/r06_occ3q/pmc_rollout.json
