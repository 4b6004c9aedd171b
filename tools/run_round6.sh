#!/bin/bash
# Round-6 validation sessions on the final tree (the in-tree build), summarised on the box into
# gpurun_out/summary/$PROFILE_TAG (copy to profiles/ afterwards):
#   PART=1  smoke, the whole -m gpu suite, the default bench line, the driver-shaped lines
#   PART=2  rocprofv3 stats of the driver's and the default command, the PMC passes of the (K = 20, K = 1 000)
#           rollout and the perft leg, and the API steps' PMC (tools/api_pmc.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${PROFILE_TAG:-r06_final}
if [ "${PART:-1}" = 1 ]; then
  PROFILE_TAG=$TAG STEPS="smoke pytest bench short" bash tools/gpu_run.sh || exit $?
else
  PROFILE_TAG=$TAG STEPS="profs prof pmcrf pmcrw pmcrm pmcrl pmcpf pmcpw pmcpm" bash tools/gpu_run.sh || exit $?
  timeout -k 10 600 bash tools/api_pmc.sh > gpurun_out/api_pmc.log 2>&1 || { echo "api_pmc rc=$?"; tail -5 gpurun_out/api_pmc.log; exit 7; }
  mkdir -p gpurun_out/summary/$TAG && cp gpurun_out/pmc_api.json gpurun_out/summary/$TAG/pmc_api.json
  tail -3 gpurun_out/api_pmc.log
fi
echo ROUND6DONE
