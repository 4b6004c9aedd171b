"""Diagnostic: per-call latency of the drop-in ChessEngine's four methods on one state dict
(the reference env calls them once or twice per step: chess_v2.py:204, 419, 579, 590), split
into the Python conversion and the C-ABI call.

    python tools/engine_probe.py [--calls 500]      (GC_ENGINE_ZC=0: the staged copies)
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
    ap.add_argument("--calls", type=int, default=500)
    a = ap.parse_args()
    from gym_chess_amd import codec as C
    from gym_chess_amd.engine import ChessEngine

    eng = ChessEngine(0)
    state = dict(board=C.DEFAULT_BOARD, current_player="WHITE", white_king_castle_is_possible=True,
                 white_queen_castle_is_possible=True, black_king_castle_is_possible=True,
                 black_queen_castle_is_possible=True)
    ops = {
        "get_possible_moves": lambda: eng.get_possible_moves(state, "WHITE"),
        "get_possible_moves_attack": lambda: eng.get_possible_moves(state, "WHITE", True),
        "get_castle_moves": lambda: eng.get_castle_moves(state, "WHITE"),
        "next_state": lambda: eng.next_state(state, "WHITE", "e2e4"),
        "update_state": lambda: eng.update_state(state),
        "dict_to_arrays (host only)": lambda: C.dict_to_arrays(state),
    }
    out = {"zero_copy": os.environ.get("GC_ENGINE_ZC", "1") != "0", "calls": a.calls, "us_per_call": {}}
    for name, f in ops.items():
        for _ in range(20):
            f()
        t0 = time.perf_counter()
        for _ in range(a.calls):
            f()
        out["us_per_call"][name] = (time.perf_counter() - t0) / a.calls * 1e6
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
