#!/bin/bash
# Round-6 validation at scale, second session (the final code, all against the oracle): fused
# rollouts in 2 000-ply (k_env_rollout4<true>) and 599-ply (<false>) launches, the quad API step
# and the random opponent's API step for both colours over 20 000 steps, FIDE fused rollouts
# against the host build of gc_fide.h
#   /usr/local/graft/bin/gpurun --timeout 1200 -- bash tools/validate_r06b.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/val
timeout -k 10 600 python -u tools/soak.py --plies 20000 --chunk 2000 --seeds 4 --seed-base 12000 > gpurun_out/val/soak_fused_k2000.jsonl 2>gpurun_out/val/soak_k2000.err || exit 3
timeout -k 10 400 python -u tools/soak.py --plies 20000 --chunk 599 --seeds 2 --seed-base 15000 > gpurun_out/val/soak_fused_k599.jsonl 2>gpurun_out/val/soak_k599.err || exit 4
timeout -k 10 300 python -u tools/soak.py --api --plies 20000 --seeds 2 > gpurun_out/val/soak_api.jsonl 2>gpurun_out/val/soak_api.err || exit 5
timeout -k 10 300 python -u tools/soak.py --api-opp WHITE --plies 20000 --seeds 1 > gpurun_out/val/soak_api_opp_white.jsonl 2>gpurun_out/val/soak_api_opp_w.err || exit 6
timeout -k 10 300 python -u tools/soak.py --api-opp BLACK --plies 20000 --seeds 1 > gpurun_out/val/soak_api_opp_black.jsonl 2>gpurun_out/val/soak_api_opp_b.err || exit 7
timeout -k 10 300 python -u tools/soak.py --fide --plies 4000 --chunk 1000 --seeds 2 > gpurun_out/val/soak_fide.jsonl 2>gpurun_out/val/soak_fide.err || exit 8
echo VALIDATION_OK
