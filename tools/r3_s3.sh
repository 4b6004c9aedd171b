#!/bin/bash
# launch anatomy with wave placement (GC_PSTAMPS build): where the slow waves of the fused launch run
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
(rocminfo 2>/dev/null | grep -E "Compute Unit|SIMDs per CU|Marketing|gfx" | head -12) > gpurun_out/rocminfo.log || true
cat gpurun_out/rocminfo.log
run() { local n=$1 s=$2; shift 2; timeout -k 10 "$s" "$@" > gpurun_out/$n.log 2>&1; local rc=$?; tail -30 gpurun_out/$n.log; [ $rc -eq 0 ] || { echo "STOP $n rc=$rc"; exit $rc; }; }
run pst20 120 python tools/pstamp_probe.py 65536 20
run pst1000 120 python tools/pstamp_probe.py 65536 1000
