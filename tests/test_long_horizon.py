"""Long-horizon full-size soak inside the GPU suite: the horizon that
found round 4's two-pins bug (tools/soak.py: 65 536 boards x 20 000 plies, where no shorter
test had met the position).  Each case runs the device's random self-play as fused launches of
2 000 plies with the per-ply trace and checks every ply's action / reward / done / reason of
224 sampled boards (strided, the first / last 64, the middle 32) and their final states against
the oracle driver (oracle/gc_oracle.c restating chess_v2.py:219-294 over lib.rs).
Cases: opponent "none" (the headline kernel k_env_rollout4), the random opponent for a WHITE
agent and for a BLACK agent (whose unbounded windows go through the spill table); and the
random opponent's device API step (k_env_step_api4_vs, both colours) stepped with its own picks,
auto-reset on.
Reference: test_benchmark.py:9-43 (the driver), chess_v2.py:116-127 (the random policy),
chess_v2.py:192, 402-407 (3-fold), lib.rs:460-784 (moves, next_state)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

pytestmark = pytest.mark.gpu

N = 65536
PLIES = 20000


@pytest.mark.parametrize("seed,opp,color", [(777001, "none", "WHITE"), (777002, "random", "WHITE"),
                                            (777003, "random", "BLACK")])
def test_soak_full_size_20000_plies(oracle, seed, opp, color):
    import soak

    idx = soak.default_sample(N)
    bad, spill, secs = soak.fused_case(seed, opp, color, None, PLIES, 2000, N, idx,
                                       threads=max(1, min(16, os.cpu_count() or 1)))
    print(f"seed {seed} {opp} {color}: {len(idx)} boards x {PLIES} plies equal, spill {spill}, {secs} s")
    assert not bad, bad[:8]


@pytest.mark.parametrize("seed,color", [(778001, "WHITE"), (778002, "BLACK")])
def test_api_opponent_full_size(oracle, seed, color):
    """65 536 boards x 3 000 API steps against the random opponent, 192 sampled boards checked
    step by step (reward, done, reason, the next pick) and their states every 500 steps."""
    import numpy as np
    import soak

    idx = np.array(sorted(set(range(0, N, 1021)) | set(range(64)) | set(range(N - 64, N))), dtype=np.int64)
    bad, steps, spill, secs = soak.api_opp_case(seed, color, 3000, N, idx)
    print(f"api opponent {color} seed {seed}: {steps} board steps equal, spill {spill}, {secs} s")
    assert not bad and steps == 3000 * len(idx), bad[:8]
