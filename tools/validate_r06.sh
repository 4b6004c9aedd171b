#!/bin/bash
# Round-6 validation at scale (one gpurun session), all against the oracle: fused-rollout soaks of
# 65 536 boards x 20 000 plies in launches of 1 000 plies (k_env_rollout4<true>, the occupancy
# filter; the random opponent's cases on the paired kernel) and of 700 plies (<false>), and perft
# fuzz of mid-game positions
#   /usr/local/graft/bin/gpurun --timeout 1200 -- bash tools/validate_r06.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/val
timeout -k 10 700 python -u tools/soak.py --plies 20000 --chunk 1000 --seeds 6 --seed-base 6000 > gpurun_out/val/soak_fused_k1000.jsonl 2>gpurun_out/val/soak_k1000.err || exit 3
timeout -k 10 400 python -u tools/soak.py --plies 20000 --chunk 700 --seeds 2 --seed-base 9000 > gpurun_out/val/soak_fused_k700.jsonl 2>gpurun_out/val/soak_k700.err || exit 4
timeout -k 10 200 python -u tools/perft_fuzz.py --midgame --scale 2 > gpurun_out/val/perft_fuzz.log 2>&1 || exit 5
echo VALIDATION_OK
