#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
REPS=2 LIBS="tools/_lib_quad.so tools/_lib_noprobe.so tools/_lib_quad.so@GC_NO_QUAD=1 tools/_lib_noprobe.so@GC_NO_QUAD=1" bash tools/r3_ab.sh
