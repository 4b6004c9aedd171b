#!/usr/bin/env python3
"""Where the fixed cost of a short timed region goes (VERDICT r02 "next" #2).

bench.py's headline region is [sync; t0; event; step_random(K); event; sync; t1].  For
K = 20 (the driver's --steps) and K = 1000 it prints, per repeat: wall us per ply, event us
per ply, the host time to enqueue the K plies, and the host time from t0 to the end event's
completion.  Run on the GPU box:  python tools/short_probe.py [--streams 1,2] [--reps 5]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-chess_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", default="1,2")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--ks", default="20,1000")
    ap.add_argument("--boards", type=int, default=65536)
    ap.add_argument("--settle", type=int, default=1000)
    ap.add_argument("--fused", action="store_true", help="time rollout_device(K) with a per-ply trace instead")
    ap.add_argument("--no-events", action="store_true", help="fused: no event slots (wall clock only)")
    a = ap.parse_args()
    from gym_chess_amd.env import BatchedChessEnv

    env = BatchedChessEnv(a.boards, device=0, seed=0x5EED + 3)
    env.rollout(a.settle)
    env.step_random(50)
    env.synchronize()
    res = []
    tb = env.trace_buffer(max(int(x) for x in a.ks.split(","))) if a.fused else None
    if a.fused:
        env.rollout_device(5, tb)
    for s in [int(x) for x in a.streams.split(",")]:
        env.set_streams(s)
        env.step_random(5)
        env.synchronize()
        for k in [int(x) for x in a.ks.split(",")]:
            for r in range(a.reps):
                env.synchronize()
                t0 = time.perf_counter()
                if a.fused:
                    env.rollout_device(k, tb, events=(-1, -1) if a.no_events else (0, 1))
                else:
                    env.record_event(0)
                    env.step_random(k)
                    env.record_event(1)
                t_enq = time.perf_counter()
                env.synchronize()
                t1 = time.perf_counter()
                ev = 0.0 if a.no_events else env.elapsed_ms(0, 1) * 1e3
                row = {"fused": a.fused, "streams": s, "k": k, "rep": r, "wall_us_per_ply": (t1 - t0) * 1e6 / k,
                       "event_us_per_ply": ev / k, "enqueue_us": (t_enq - t0) * 1e6, "wall_us": (t1 - t0) * 1e6,
                       "event_us": ev}
                res.append(row)
                print(json.dumps({k2: (round(v, 2) if isinstance(v, float) else v) for k2, v in row.items()}),
                      flush=True)
    env.close()
    import numpy as np

    for k in sorted({r["k"] for r in res}):
        w = np.median([r["wall_us"] for r in res if r["k"] == k])
        e = np.median([r["event_us"] for r in res if r["k"] == k])
        print(f"# k={k}: median wall {w:.1f} us ({w / k:.3f}/ply), event {e:.1f} us ({e / k:.3f}/ply), "
              f"markers={'GC_MARKER_EVENTS' in os.environ}", flush=True)


if __name__ == "__main__":
    main()
