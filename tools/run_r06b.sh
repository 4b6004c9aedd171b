#!/bin/bash
# Round-6 session B: phase stamps of the baseline, the late commit and the late commit + key
# ring; parity gate and same-box A/B of the leaper / king-set role moves.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in pst pstlate pstring; do
  PST_QUAD=1 PST_LIB=tools/_lib_$v.so timeout -k 10 120 python tools/pstamp_probe.py 65536 1000 > gpurun_out/r06b_$v.log 2>&1 || { echo "PST $v rc=$?"; tail -5 gpurun_out/r06b_$v.log; exit 3; }
  echo "== $v"; cat gpurun_out/r06b_$v.log
done
PARITY=1 LIBS="gym-chess_amd/gym_chess_amd/libgymchess.so tools/_lib_kq3.so tools/_lib_lq3.so tools/_lib_klq3.so" REPS=${REPS:-3} bash tools/ab.sh || exit 4
