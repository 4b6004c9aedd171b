#!/bin/bash
# the role priorities: parity subset on this build (Q0 2, Q1 2), then same-box A/B against the
# HEAD build, the phase-3 swap (GC_QPRIO_DYN) and Q1 above Q0 (GC_QPRIO=0x0E)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
M=gym-chess_amd/gym_chess_amd/libgymchess.so
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 3; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_full_size.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1 || { tail -20 gpurun_out/pt.log; exit 3; }
tail -1 gpurun_out/pt.log
REPS=2 LIBS="tools/_lib_q12.so $M tools/_lib_prd.so tools/_lib_pre.so" bash tools/r3_ab.sh
