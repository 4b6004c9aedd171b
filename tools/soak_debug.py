"""Diagnostic: one board's divergence from the oracle found by tools/soak.py, under three
driver forms (fused launches in chunks, one fused launch, launched plies), with the states
around the first divergent ply.

    python tools/soak_debug.py SEED BOARD PLY [--chunk 2000]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gym-chess_amd"), os.path.join(ROOT, "oracle")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("seed", type=int)
    ap.add_argument("board", type=int)
    ap.add_argument("ply", type=int)
    ap.add_argument("--chunk", type=int, default=2000)
    ap.add_argument("--boards", type=int, default=65536)
    a = ap.parse_args()
    import oracle as O
    from gym_chess_amd import codec as C
    from gym_chess_amd.env import BatchedChessEnv

    i, P = a.board, a.ply
    span = P + 12
    ref = O.rollout_trace(a.seed, i, span)
    for form in ("chunks", "one", "launched"):  # (GC_NO_QUAD=1 in the environment: the paired fused kernel)
        env = BatchedChessEnv(a.boards, device=0, seed=a.seed)
        tb = env.trace_buffer(max(a.chunk, span))
        got = []
        if form == "launched":
            for p in range(span):
                env.step_random(1)
                o = env.outputs()
                got.append((int(o["reward"][i]), int(o["done"][i]), int(o["reason"][i])))
            acts = None
        else:
            step = a.chunk if form == "chunks" else span
            acts, rws, dns, why = [], [], [], []
            for p in range(0, span, step):
                k = min(step, span - p)
                env.rollout_device(k, tb)
                env.synchronize()
                tr = tb.fetch(k)
                acts += list(tr["action"][:, i]); rws += list(tr["reward"][:, i])
                dns += list(tr["done"][:, i]); why += list(tr["reason"][:, i])
            got = list(zip(rws, dns, why))
        first = None
        for p in range(span):
            w = (int(ref["reward"][p]), int(ref["done"][p]), int(ref["reason"][p]))
            g = (int(got[p][0]), int(got[p][1]), int(got[p][2]))
            if g != w or (acts is not None and int(acts[p]) != int(ref["action"][p])):
                first = p
                break
        print(f"[{form}] first divergence at ply {first}", flush=True)
        if first is not None and acts is not None:
            lo = max(0, first - 6)
            print("  oracle actions", [int(x) for x in ref["action"][lo:first + 3]])
            print("  device actions", [int(x) for x in acts[lo:first + 3]])
            print("  oracle reward/done/reason", [(int(ref["reward"][p]), int(ref["done"][p]), int(ref["reason"][p]))
                                                  for p in range(lo, first + 3)])
            print("  device reward/done/reason", [tuple(int(v) for v in got[p]) for p in range(lo, first + 3)])
            pre = O.rollout_trace(a.seed, i, first)  # the state before the divergent ply
            b, m = pre["final_board"], pre["final_meta"]
            print("  oracle state before it: meta", list(m))
            print(C.board_to_text(b))
            lst = O.get_possible_moves(b, m, int(m[0]))
            print("  oracle legal list", len(lst), lst[:60])
        tb.close()
        env.close()


if __name__ == "__main__":
    main()
