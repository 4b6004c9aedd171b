#!/usr/bin/env python3
"""configs[3] at full width: the bench's 65 536 mid-game perft roots and their node counts,
computed by the C oracle (oracle/gc_oracle.c -- test infrastructure), committed as
tests/golden/configs3_perft.npz.

The roots are regenerated exactly as bench.py's `midgame_fens` makes them on the device:
board i is the position after 10 + (i*7919 mod 31) plies of the random self-play driver
(seed 0x5EED + 4, replica 0; the oracle's `rollout_trace` restates that driver per board --
tests/test_full_size.py pins it against the device), exported to FEN (board, side, the four
stored castle rights; no check flags) and read back, then `update_state` (chess_v2.py:204)
fills the check flags.  Perft is the reference's by composition (lib.rs:460-486 move lists,
679-784 next_state, the rights re-read by State::new 295-336 at every node).

Stored (data only):
  boards   int8[65536, 64]   the roots (row 0 = rank 8, lib.rs:41-50)
  metas    uint8[65536, 8]   {white_to_move, wkc, wqc, bkc, bqc, wchk, bchk, move_count}
  perft4   uint64[65536]     perft(4) of every root
  stride5  int64[1024]       root indices 0, 64, 128, ... (every 64th root)
  perft5   uint64[1024]      perft(5) of those roots

Usage: python tests/golden/make_perft_roots.py [--threads 8] [--work /tmp/perft_roots]
(about 7e10 + 4e10 oracle nodes: tens of minutes on 8 cores; partial results are kept in
--work so an interrupted run resumes).
"""
import argparse
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))

import oracle as O  # noqa: E402

N = 65536
SEED = 0x5EED + 4  # bench.py perft_leg: rp.board_seed(0x5EED + 4), replica 0
STRIDE5 = 64
OUT = os.path.join(HERE, "configs3_perft.npz")


def root_plies(n=N):
    """bench.py midgame_fens: board i is taken after 10 + (i*7919 mod 31) plies"""
    return 10 + (np.arange(n, dtype=np.int64) * 7919) % 31


def make_roots(threads, n=N, seed=SEED):
    ply = root_plies(n)

    def one(i):
        r = O.rollout_trace(seed, int(i), int(ply[i]))
        m = np.zeros(8, np.uint8)
        m[:5] = r["final_meta"][:5]  # the FEN keeps side + the four stored rights
        m[7] = r["final_meta"][7]    # full-move number n <-> move_count n - 1
        b, mm = O.update_state(r["final_board"], m)
        mm[7] = m[7]
        return b, mm

    with ThreadPoolExecutor(threads) as ex:
        res = list(ex.map(one, range(n)))
    return np.stack([r[0] for r in res]), np.stack([r[1] for r in res])


def perft_chunked(boards, metas, depth, threads, work, tag, chunk=2048):
    os.makedirs(work, exist_ok=True)
    out = np.zeros(len(boards), np.uint64)
    t0 = time.time()
    for lo in range(0, len(boards), chunk):
        f = os.path.join(work, f"{tag}_{lo}.npy")
        if os.path.exists(f):
            out[lo:lo + chunk] = np.load(f)
            continue
        v = O.perft_batch(boards[lo:lo + chunk], metas[lo:lo + chunk], depth, threads)
        np.save(f, v)
        out[lo:lo + chunk] = v
        print(f"{tag}: {lo + len(v)}/{len(boards)} roots, {time.time() - t0:.0f} s", flush=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 8)
    ap.add_argument("--work", default="/tmp/perft_roots")
    args = ap.parse_args()
    O.lib()
    t0 = time.time()
    boards, metas = make_roots(args.threads)
    print(f"roots: {time.time() - t0:.1f} s", flush=True)
    s5 = np.arange(0, N, STRIDE5, dtype=np.int64)
    p4 = perft_chunked(boards, metas, 4, args.threads, args.work, "p4")
    p5 = perft_chunked(boards[s5], metas[s5], 5, args.threads, args.work, "p5", chunk=64)
    np.savez_compressed(OUT, boards=boards, metas=metas, perft4=p4, stride5=s5, perft5=p5)
    print(f"wrote {OUT}: perft4 total {int(p4.sum())}, perft5 stride total {int(p5.sum())}, "
          f"{time.time() - t0:.0f} s", flush=True)


if __name__ == "__main__":
    main()
