"""Diagnostic: per-ply step_random outputs vs the oracle driver; first divergence."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-chess_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402
from gym_chess_amd.env import BatchedChessEnv  # noqa: E402

n, seed, plies = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
env = BatchedChessEnv(n, device=0, seed=seed)
refs = [O.rollout_trace(seed, i, plies + 1) for i in range(n)]
ra = np.stack([r["action"] for r in refs], axis=1)
for p in range(plies):
    env.step_random(1)
    o = env.outputs()
    nxt = np.where(ra[p + 1] < 0, 0xFFFF, ra[p + 1]).astype(np.uint16)
    bad = np.nonzero(o["next_action"] != nxt)[0]
    rr = np.stack([r["reward"][p] for r in refs])
    badr = np.nonzero(o["reward"] != rr)[0]
    if len(bad) or len(badr):
        i = int(bad[0]) if len(bad) else int(badr[0])
        print("ply", p, "boards", bad[:10], badr[:10], "gpu", o["next_action"][i], "oracle", nxt[i],
              "gpu rw", o["reward"][i], "oracle rw", rr[i], "reason", o["reason"][i], refs[i]["reason"][p])
        print("oracle actions", ra[max(0, p - 5):p + 2, i])
        b, m = env.boards()
        print("meta", m[i])
        print(b[i].reshape(8, 8))
        break
else:
    print("no divergence")
