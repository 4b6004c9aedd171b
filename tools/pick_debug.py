"""Diagnostic: first plies of step_random vs the oracle; for mismatched boards print the
position, both picks and the legal actions in action-id order."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-chess_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402
from gym_chess_amd import codec as C  # noqa: E402
from gym_chess_amd.env import BatchedChessEnv  # noqa: E402

n, seed, plies = 64, 777, 3
env = BatchedChessEnv(n, device=0, seed=seed)
refs = [O.rollout_trace(seed, i, plies + 1) for i in range(n)]
for p in range(plies):
    env.step_random(1)
    o = env.outputs()
    b, m = env.boards()
    for i in range(n):
        want = refs[i]["action"][p + 1]
        if int(o["next_action"][i]) != int(want) % 65536:
            acts = sorted(O.get_possible_moves(b[i], m[i], int(m[i, 0])))
            print("ply", p, "board", i, "gpu", o["next_action"][i], C.action_to_str(o["next_action"][i]),
                  "oracle", want, C.action_to_str(want), "n legal", len(acts),
                  "gpu rank", acts.index(int(o["next_action"][i])) if int(o["next_action"][i]) in acts else None,
                  "oracle rank", acts.index(int(want)) if int(want) in acts else None)
            print(C.board_to_text(b[i]), m[i])
