"""Diagnostic: one configs[1]-shaped perft call (4 096 start positions, perft(3), through the
engine C-ABI) repeated, for rocprofv3's kernel / copy traces of where a call's time goes:
  rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/pcp -o run -- python tools/perft_call_probe.py"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-chess_amd"))
from gym_chess_amd import _lib  # noqa: E402
from gym_chess_amd import codec as C  # noqa: E402
from gym_chess_amd.engine import Engine  # noqa: E402

if os.environ.get("PCP_LIB"):  # another build (A/B)
    _lib.load(os.path.abspath(os.environ["PCP_LIB"]))

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
b = np.tile(np.asarray(C.DEFAULT_BOARD, np.int8).reshape(1, 64), (n, 1))
m = np.zeros((n, 8), np.uint8)
m[:, 0:5] = 1
eng = Engine(0)
r0 = eng.perft(b, m, 3)
print("first call: nodes per root", np.unique(r0)[:4], int(r0.sum()))
calls = int(os.environ.get("PCP_CALLS", "20"))
bad = 0
t0 = time.perf_counter()
for _ in range(calls):
    r = eng.perft(b, m, 3)
    bad += int((r != 8982).any())  # (the reference rules' perft(3) of the start position)
dt = (time.perf_counter() - t0) / calls
print(f"calls {calls}, calls with a wrong root {bad}")
print("nodes per root", np.unique(r)[:4], int(r.sum()))
print(f"{n} roots perft(3): {dt * 1e3:.3f} ms per call")
eng.close()
