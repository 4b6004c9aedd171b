"""Diagnostic only: parity gate for an A/B build of libgymchess.so -- the fused rollout's
per-ply trace (opponent none, random opponent WHITE / BLACK agent) and the launched step's
final states, against the oracle, before its timing is trusted.

    python tools/ab_parity.py tools/_lib_<tag>.so
"""
import os
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gym-chess_amd"), os.path.join(ROOT, "oracle")]
from gym_chess_amd import _lib  # noqa: E402

_lib.load(os.path.abspath(sys.argv[1]))
import oracle as O  # noqa: E402
from gym_chess_amd.env import BatchedChessEnv  # noqa: E402

n, plies = 320, 400
for seed, kw, okw in ((11, {}, {}), (12, dict(opponent="random"), dict(opponent=1)),
                      (13, dict(opponent="random", player_color="BLACK"), dict(opponent=1, agent_white=False))):
    env = BatchedChessEnv(n, device=0, seed=seed, **kw)
    tb = env.trace_buffer(plies)
    env.rollout_device(plies, tb)
    tr = tb.fetch()
    launched = BatchedChessEnv(n, device=0, seed=seed, **kw)
    launched.step_random(plies)
    with ThreadPoolExecutor(16) as ex:
        refs = list(ex.map(lambda i: O.rollout_trace(seed, i, plies, **okw), range(n)))
    b, m = launched.boards()
    for i, r in enumerate(refs):
        for k in ("action", "reward", "done", "reason"):
            assert (tr[k][:, i] == r[k]).all(), (kw, i, k)
        assert (b[i] == r["final_board"]).all() and list(m[i]) == list(r["final_meta"]), (kw, i)
    print("parity ok", kw or "opponent none", flush=True)
