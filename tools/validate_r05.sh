# Round-5 validation at scale (one gpurun session): 6 fused-rollout soaks + both opponent colours at
# 65 536 boards x 20 000 plies, the quad opponent API step (WHITE) and the quad API step over
# 20 000 steps, perft fuzz of mid-game positions -- all against the oracle
#   /usr/local/graft/bin/gpurun --timeout 1200 -- bash tools/validate_r05.sh
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/val
timeout -k 10 700 python -u tools/soak.py --plies 20000 --chunk 2000 --seeds 6 > gpurun_out/val/soak_fused.jsonl 2>gpurun_out/val/soak_fused.err || exit 3
timeout -k 10 300 python -u tools/soak.py --api-opp WHITE --plies 20000 --seeds 1 > gpurun_out/val/soak_api_opp_white.jsonl 2>gpurun_out/val/soak_api_opp.err || exit 4
timeout -k 10 200 python -u tools/soak.py --api --plies 20000 --seeds 2 > gpurun_out/val/soak_api.jsonl 2>gpurun_out/val/soak_api.err || exit 5
timeout -k 10 200 python -u tools/perft_fuzz.py --midgame --scale 2 > gpurun_out/val/perft_fuzz.log 2>&1 || exit 6
echo VALIDATION_OK
