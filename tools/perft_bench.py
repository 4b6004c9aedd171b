"""Perft throughput probe: configs[1] (4096 startpos x perft(3)) and configs[3]-shaped
mid-game roots (random self-play positions) x perft(d)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-chess_amd"))
from gym_chess_amd.engine import Engine  # noqa: E402
from gym_chess_amd.env import BatchedChessEnv  # noqa: E402

eng = Engine(0)
start = np.array([-3, -5, -4, -2, -1, -4, -5, -3] + [-6] * 8 + [0] * 32 + [6] * 8 + [3, 5, 4, 2, 1, 4, 5, 3], np.int8)
b = np.tile(start, (4096, 1))
m = np.tile(np.array([1, 1, 1, 1, 1, 0, 0, 0], np.uint8), (4096, 1))
for d in (3, 4):
    t = time.perf_counter()
    r = eng.perft(b, m, d)
    dt = time.perf_counter() - t
    print(f"startpos x4096 perft({d}) = {int(r[0])} each, {r.sum():.3e} nodes, {dt:.3f} s, {r.sum()/dt:.3e} nodes/s", flush=True)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
depth = int(sys.argv[2]) if len(sys.argv) > 2 else 5
env = BatchedChessEnv(n, device=0, seed=0x5EED + 4)
env.step_random(25)
bb, mm = env.boards()
for d in range(1, depth + 1):
    t = time.perf_counter()
    r = eng.perft(bb, mm, d)
    dt = time.perf_counter() - t
    print(f"midgame x{n} perft({d}): {r.sum():.4e} nodes, {dt:.3f} s, {r.sum()/dt:.3e} nodes/s", flush=True)
