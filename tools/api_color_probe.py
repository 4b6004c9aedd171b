"""Diagnostic only: the random opponent's API step per launch (HIP events) for a WHITE and a
BLACK agent, quad (k_env_step_api4_vs) and paired (GC_NO_QUAD_API=1) kernels, 65 536 boards.

    python tools/api_color_probe.py [boards] [steps]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-chess_amd"))
from gym_chess_amd.env import BatchedChessEnv  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 300
for color in ("WHITE", "BLACK"):
    for paired in (False, True):
        if paired:
            os.environ["GC_NO_QUAD_API"] = "1"
        env = BatchedChessEnv(n, device=0, seed=99, opponent="random", player_color=color)
        env.rollout(200)
        io = env.device_io()
        for _ in range(20):
            env.step_device(io, autoreset=True)
        env.record_event(4)
        for _ in range(steps):
            env.step_device(io, autoreset=True)
        env.record_event(5)
        env.synchronize()
        us = env.elapsed_ms(4, 5) * 1e3 / steps
        print(f"{color} {'paired' if paired else 'quad'}: {us:.2f} us per launch, {n / us / 1e3:.3f}e9 env.steps/s")
        io.close()
        env.close()
        os.environ.pop("GC_NO_QUAD_API", None)
