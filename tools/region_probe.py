"""Diagnostic only: bench.py's headline timed region ([sync; t0; rollout_device(K) with events;
sync; t1]) repeated in one process, the first region separately -- what a cold first call
costs (event slots never recorded before, cold host paths).
    python tools/region_probe.py [--warm-events] [--k 20] [--reps 6]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-chess_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--warm-events", action="store_true")
    ap.add_argument("--k", type=int, default=20)
    ap.add_argument("--reps", type=int, default=6)
    a = ap.parse_args()
    from gym_chess_amd.env import BatchedChessEnv

    env = BatchedChessEnv(65536, device=0, seed=0x5EED + 3)
    env.rollout(1000)
    tb = env.trace_buffer(max(a.k, 5))
    env.rollout_device(5, tb, events=(0, 1) if a.warm_events else (-1, -1))
    env.synchronize()
    if a.warm_events:
        env.elapsed_ms(0, 1)
    out = []
    for r in range(a.reps):
        env.synchronize()
        t0 = time.perf_counter()
        env.rollout_device(a.k, tb, events=(0, 1))
        t1 = time.perf_counter()
        env.synchronize()
        t2 = time.perf_counter()
        out.append({"rep": r, "wall_us": round((t2 - t0) * 1e6, 1), "enqueue_us": round((t1 - t0) * 1e6, 1),
                    "event_us": round(env.elapsed_ms(0, 1) * 1e3, 1)})
    print(json.dumps({"warm_events": a.warm_events, "k": a.k, "regions": out}), flush=True)


if __name__ == "__main__":
    main()
