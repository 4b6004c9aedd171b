#!/bin/bash
# Instruction mix of one kernel in the gfx950 ISA of gymchess.hip (diagnostic).
#   tools/isa_stats.sh <mangled-kernel-name> [src.hip]
K=${1:-_Z11k_env_step26EnvDev}
SRC=${2:-$(dirname $0)/../gym-chess_amd/csrc/gymchess.hip}
T=$(mktemp -d)
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-discard-value-names -S --cuda-device-only -o $T/k.s "$SRC" 2>/dev/null
awk -v k="$K:" '$1==k{on=1} on{print} on && /^\.Lfunc_end/{exit}' $T/k.s > $T/kern.s
echo "lines $(wc -l < $T/kern.s)  branches $(grep -c 's_cbranch' $T/kern.s)  saveexec $(grep -c 's_and_saveexec' $T/kern.s)  valu $(grep -c '^\s*v_' $T/kern.s)  salu $(grep -c '^\s*s_' $T/kern.s)"
cp $T/kern.s /tmp/kern_last.s
rm -rf $T
