#!/bin/bash
# round-3 session: parity, launch anatomy (GC_PSTAMPS build), short-region probe with the
# fused launch timed by its own dispatch events vs marker events vs none, driver-shaped bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS="smoke pytest" bash tools/gpu_run.sh || exit $?
run() { local n=$1 s=$2; shift 2; timeout -k 10 "$s" "$@" > gpurun_out/$n.log 2>&1; local rc=$?; tail -12 gpurun_out/$n.log; [ $rc -eq 0 ] || { echo "STOP $n rc=$rc"; exit $rc; }; }
run pst20 120 python tools/pstamp_probe.py 65536 20
run pst1000 120 python tools/pstamp_probe.py 65536 1000
run sp_ext 200 python tools/short_probe.py --fused --streams 1 --ks 5,10,20,40,1000 --reps 5
GC_MARKER_EVENTS=1 run sp_mark 200 python tools/short_probe.py --fused --streams 1 --ks 5,10,20,40,1000 --reps 5
run sp_none 200 python tools/short_probe.py --fused --no-events --streams 1 --ks 5,10,20,40,1000 --reps 5
STEPS="short" PROFILE_TAG=${PROFILE_TAG:-r03_v4} bash tools/gpu_run.sh
