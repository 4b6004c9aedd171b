#!/bin/bash
# one round-3 profile set of the current build: parity, smoke, the default bench line, the
# driver's command three times plus a long line, rocprof stats of both, PMC of the headline
# and of the perft leaf
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
STEPS="smoke pytest bench short prof profs pmcrf pmcrw pmcrm pmcpf pmcpw pmcpm" PROFILE_TAG=${PROFILE_TAG:-r03_v11} bash tools/gpu_run.sh
