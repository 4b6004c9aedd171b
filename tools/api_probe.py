"""Diagnostic: per-launch time of the API-shaped device step (k_env_step_api) by output set."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-chess_amd"))
from gym_chess_amd.env import BatchedChessEnv  # noqa: E402

n = 65536
for tag, kw in (("all", {}), ("no-mask", dict(mask=False)), ("no-obs", dict(obs=False)),
                ("pick-only", dict(mask=False, obs=False, count=False))):
    env = BatchedChessEnv(n, device=0, seed=11)
    env.rollout(500)
    io = env.device_io(**kw)
    for _ in range(20):
        env.step_device(io, autoreset=True)
    env.synchronize()
    env.record_event(4)
    K = 200
    for _ in range(K):
        env.step_device(io, autoreset=True)
    env.record_event(5)
    env.synchronize()
    print(tag, "%.2f us per launch" % (env.elapsed_ms(4, 5) * 1e3 / K))
    io.close()
    env.close()
