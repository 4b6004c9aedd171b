"""Diagnostic only: where one quad API step (k_env_step_api4; with "vs": k_env_step_api4_vs, its
seven phases' work and the entry + waits together) spends its time, per role -- the
cycles of each segment (entry loads, phase 0, wait A, phase 1, wait B, phase 2, wait C,
phase 3 with its stores; s_memtime) and the launch anatomy (wave start / end on the 100 MHz
clock).  Build: tools/build_variants.sh pst "-DGC_PSTAMPS" -> tools/_lib_pst.so.

    python tools/api_pstamp_probe.py [boards] [steps before the stamped one] [vs]
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-chess_amd"))
from gym_chess_amd import _lib  # noqa: E402

L = _lib.load(os.environ.get("PST_LIB") or os.path.join(ROOT, "tools", "_lib_pst.so"))
L.gc_debug_api_pstamps.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
from gym_chess_amd.env import BatchedChessEnv  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
warm = int(sys.argv[2]) if len(sys.argv) > 2 else 100
vs = len(sys.argv) > 3 and sys.argv[3] == "vs"  # the random opponent's quad step (k_env_step_api4_vs)
env = BatchedChessEnv(n, device=0, seed=0x5EED + 14, **({"opponent": "random"} if vs else {}))
env.rollout(1000)
io = env.device_io()
for _ in range(warm):
    env.step_device(io, autoreset=True)
env.synchronize()
waves = ((n + 127) // 128) * 8
out = np.zeros(waves * 12, dtype=np.uint64)
rows = []
for rep in range(5):
    _lib.check(L.gc_debug_api_pstamps(env._h, 1, None))
    env.step_device(io, autoreset=True)
    _lib.check(L.gc_debug_api_pstamps(env._h, 0, out.ctypes.data))
    rows.append(out.reshape(-1, 12).copy())
raw = np.concatenate(rows)
st = raw[:, :8].astype(np.float64)
rt = (raw[:, 8:] & np.uint64((1 << 56) - 1)).astype(np.int64).reshape(5, waves, 4)
for k in range(5):
    t0 = rt[k, :, 0].min()
    us = (rt[k] - t0) / 100.0
    if k == 4:
        print(f"launch anatomy (us from the first wave's start): last wave start {us[:, 0].max():.2f}; entry loads "
              f"mean {(us[:, 1] - us[:, 0]).mean():.2f}; phases 0-2 mean {(us[:, 2] - us[:, 1]).mean():.2f}; phase 3 "
              f"mean {(us[:, 3] - us[:, 2]).mean():.2f}; wave end mean {us[:, 3].mean():.2f}, p90 "
              f"{np.percentile(us[:, 3], 90):.2f}, max {us[:, 3].max():.2f}")
w = np.arange(len(raw)) % 8
role = (w & 3) ^ (((w >> 2) & 1) << 1)
names = ["phase 0", "wait A", "phase 1", "wait B", "phase 2", "wait C", "phase 3", "entry"]
if vs:  # k_env_step_api4_vs: seven phases' work, the entry loads and every barrier wait together
    names = [f"phase {k}" for k in range(7)] + ["entry+waits"]
for r in range(4):
    s = st[role == r]
    tot = s.sum(axis=1).mean()
    print(f"[Q{r}] {len(s)} waves, {tot:.0f} cycles")
    for k in (7, 0, 1, 2, 3, 4, 5, 6):
        print(f"   {names[k]:>8}: {s[:, k].mean():7.0f}  ({s[:, k].mean() / tot:5.1%})")
