#!/bin/bash
# same-box A/B: phases 1-2 priorities (Q2 / Q3 above Q0 / Q1: m1; all equal: m2) against HEAD
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
REPS=2 LIBS="tools/_lib_q13.so tools/_lib_m1.so tools/_lib_m2.so" bash tools/r3_ab.sh
