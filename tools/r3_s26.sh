#!/bin/bash
# same-box A/B: wave priority for Q1 (GC_QPRIO=2) or Q0 + Q1 (3) against the HEAD build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
REPS=2 LIBS="tools/_lib_q12.so tools/_lib_pr2.so tools/_lib_pr3.so" bash tools/r3_ab.sh
