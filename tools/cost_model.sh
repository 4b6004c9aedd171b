#!/bin/bash
# Diagnostic only: static VALU / SALU / branch counts of each gc_core function
# (tools/cost_model.hip, one tiny kernel per function; loop bodies count once).
D=$(cd "$(dirname "$0")" && pwd)
T=$(mktemp -d)
hipcc --offload-arch=gfx950 -O3 -std=c++17 -S --cuda-device-only -o "$T/cost.s" "$D/cost_model.hip" || exit 1
for k in c_side_attacks c_gen_base c_gen_pins c_gen_enemy c_sq_attacked c_apply_legal c_board_key c_philox \
         c_gen_moves_a c_gen_moves_b c_select_action c_count_moves c_gen_init c_child_count c_count_position; do
    awk -v k="$k:" '$1==k{on=1} on{print} on && /s_endpgm/{exit}' "$T/cost.s" > "$T/f.s"
    printf "%-16s valu %4d (half-rate: b64 shift/add %3d, bcnt %3d, bfrev %3d, vop3-logic %3d)  salu %4d  branches %3d  loops %d\n" \
        "$k" "$(grep -c '^\s*v_' "$T/f.s")" "$(grep -c 'v_lsh[lr]rev_b64\|v_lshl_add_u64' "$T/f.s")" \
        "$(grep -c 'v_bcnt' "$T/f.s")" "$(grep -c 'v_bfrev' "$T/f.s")" \
        "$(grep -c 'v_bitop3\|v_or3\|v_and_or\|v_bfi\|v_lshl_or' "$T/f.s")" \
        "$(grep -c '^\s*s_' "$T/f.s")" "$(grep -c 's_cbranch' "$T/f.s")" "$(grep -c 'Loop Header' "$T/f.s")"
done
rm -rf "$T"
