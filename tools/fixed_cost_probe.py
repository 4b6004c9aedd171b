"""Diagnostic only: the fixed cost of bench.py's timed region.

For K in a sweep, the headline region [sync; t0; rollout_device(K, trace, events); sync; t1]
repeated, median wall / enqueue / event time per K, with and without the two event records,
plus the bare ctypes round trip -- then the fits wall = a + b K and event = a' + b K, so
a - a' is the host's share of the fixed cost and a' the launch's (dispatch ramp, entry loads,
tail).

    python tools/fixed_cost_probe.py [path/to/libgymchess.so] [--reps 9]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-chess_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib", nargs="?", default=None)
    ap.add_argument("--reps", type=int, default=9)
    ap.add_argument("--ks", default="1,2,5,10,20,40,100")
    a = ap.parse_args()
    from gym_chess_amd import _lib

    if a.lib:
        _lib.load(os.path.abspath(a.lib))
    from gym_chess_amd.env import BatchedChessEnv

    ks = [int(k) for k in a.ks.split(",")]
    env = BatchedChessEnv(65536, device=0, seed=0x5EED + 3)
    env.rollout(1000)
    tb = env.trace_buffer(max(ks))
    env.rollout_device(5, tb, events=(0, 1))
    env.synchronize()
    env.elapsed_ms(0, 1)
    L = env._L
    t = []
    for _ in range(200):
        t0 = time.perf_counter()
        L.gc_env_num_boards(env._h)
        t.append(time.perf_counter() - t0)
    out = {"ctypes_call_us": float(np.median(t)) * 1e6, "k": {}}
    for ev, wait in ((True, "sync"), (True, "word"), (False, "sync")):
        rows = {}
        for k in ks:
            wall, enq, evt = [], [], []
            for _ in range(a.reps):
                env.synchronize()
                t0 = time.perf_counter()
                env.rollout_device(k, tb, events=(0, 1) if ev else (-1, -1))
                t1 = time.perf_counter()
                env.synchronize() if wait == "sync" else env.wait_rollout()
                t2 = time.perf_counter()
                env.synchronize()
                wall.append(t2 - t0)
                enq.append(t1 - t0)
                if ev:
                    evt.append(env.elapsed_ms(0, 1) / 1e3)
            rows[k] = {"wall_us": float(np.median(wall)) * 1e6, "enqueue_us": float(np.median(enq)) * 1e6,
                       "event_us": float(np.median(evt)) * 1e6 if evt else None}
        kk = np.array(ks, dtype=np.float64)
        wl = np.array([rows[k]["wall_us"] for k in ks])
        fit = np.polyfit(kk, wl, 1)
        res = {"rows": rows, "wall_fit": {"per_k_us": fit[0], "fixed_us": fit[1]}}
        if ev:
            el = np.array([rows[k]["event_us"] for k in ks])
            fe = np.polyfit(kk, el, 1)
            res["event_fit"] = {"per_k_us": fe[0], "fixed_us": fe[1]}
        out["k"][("events" if ev else "no_events") + "_" + wait] = res
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
