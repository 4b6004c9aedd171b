"""Diagnostic: perft of random (also weird) positions on the GPU against the oracle --
3 000 at depth 3, 400 at depth 4, 40 at depth 5 (tests/conftest.py random_positions) --
and, with --midgame, of game positions: the boards of a device self-play rollout after
10..400 plies (castling rights, checks, long games), 2 000 at depth 3 and 300 at depth 4.
--scale K multiplies the counts and draws other seeds.

    python tools/perft_fuzz.py [--scale 1] [--midgame]
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path[:0] = ["tests", "oracle", "gym-chess_amd"]
from conftest import random_positions  # noqa: E402
import oracle as O  # noqa: E402
from gym_chess_amd.engine import Engine  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--scale", type=int, default=1)
ap.add_argument("--midgame", action="store_true")
a = ap.parse_args()
eng = Engine(0)
bad = 0


def check(label, b, m, d):
    global bad
    t = time.time()
    got = eng.perft(b, m, d)
    ref = O.perft_batch(b, m, d, threads=16)
    nb = int((got != ref).sum())
    bad += nb
    print(f"{label}: {len(b)} positions perft({d}) mismatches {nb} nodes {int(ref.sum())} ({time.time()-t:.1f}s)",
          flush=True)


off = 0 if a.scale == 1 else 1000 * a.scale
for seed, n, d in ((501, 3000, 3), (502, 400, 4), (503, 40, 5)):
    b, m = random_positions(n * a.scale, seed + off)
    check(f"seed {seed + off}", b, m, d)
if a.midgame:
    from gym_chess_amd.env import BatchedChessEnv

    for seed, n, d, plies in ((601, 2000, 3, (10, 40, 120, 400)), (602, 300, 4, (10, 40, 120))):
        for p in plies:
            env = BatchedChessEnv(n * a.scale, device=0, seed=seed + off + p)
            env.rollout(p)
            b, m = env.boards()
            env.close()
            check(f"midgame seed {seed + off + p} after {p} plies", np.ascontiguousarray(b), np.ascontiguousarray(m), d)
sys.exit(1 if bad else 0)
