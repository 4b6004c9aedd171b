"""Diagnostic only: where one single-board env step goes.  Times the bare
C-ABI op (gc_env_single_call SYNC: the server round trip + the move list), the AGENT op inside
the reference driver (DeviceBoard.call), and the driver's whole step, on the device and -- the
same driver and env class -- over the C oracle's ops.
    python tools/single_probe.py [--steps 1000]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gym-chess_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"), ROOT]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=1000)
    a = ap.parse_args()
    import numpy as np

    import bench
    from gym_chess_amd.single import ChessEnv, DeviceBoard
    from oracle_engine import OracleBoard

    out = {}
    for name, mk in (("device", lambda: None), ("oracle", OracleBoard)):
        be = mk()
        env = ChessEnv(opponent="none", log=False, backend=be)
        b = env._b
        spent = [0.0]
        orig = b.call

        def timed_call(op, action=0, flags=0, _o=orig):
            t0 = time.perf_counter()
            r = _o(op, action, flags)
            spent[0] += time.perf_counter() - t0
            return r

        b.call = timed_call
        bench.reference_driver(env, 2, 100, 1)
        spent[0] = 0.0
        n, dt = bench.reference_driver(env, 10, 100, 0x5EED)
        res = {"step_us": dt / n * 1e6, "op_us": spent[0] / n * 1e6, "steps": n}
        if isinstance(b, DeviceBoard):
            import ctypes

            st = np.zeros(6, dtype=np.uint32)
            acc = np.zeros(6)
            for _ in range(200):  # AGENT ops of a fresh game: the server's segments
                acts = env.possible_actions
                if not acts:
                    env.reset()
                    continue
                env.step(acts[len(acts) // 2])
                b._L.gc_env_single_stamps(b._h, st.ctypes.data_as(ctypes.c_void_p))
                acc += st
                if env.done:
                    env.reset()
            res["server_segments_us"] = dict(zip(("request_validate", "begin", "list", "end", "record_copy", "idle_wait"), (acc / 200 / 100).tolist()))
            t = []
            for _ in range(500):
                t0 = time.perf_counter()
                orig(4)  # SYNC: round trip + the list
                t.append(time.perf_counter() - t0)
            res["sync_op_us"] = float(np.median(t)) * 1e6
        out[name] = res
        env.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
