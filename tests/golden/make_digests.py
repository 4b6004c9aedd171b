"""Generate tests/golden/full_width_digests.npz: the oracle's per-board trajectory digests of
65 536 boards x 2 000 plies of random self-play, for the headline driver (opponent "none") and
the random opponent with a WHITE and with a BLACK agent (long-horizon
parity at full width, not on a sample).

Each digest folds every ply's outputs (action, reward, done, reason; packed as the device's
trace word) and the final state of one board (oracle/gc_oracle.c oracle_rollout_digests,
restating test_benchmark.py:9-43's driver over chess_v2.py:183-294 and lib.rs:460-784).
tests/test_full_width_digest.py computes the same digest from the device's fused rollouts and
compares all 65 536 boards; its CPU part regenerates a strided sample here to pin the fixture to
the current oracle.

    python tests/golden/make_digests.py [--threads 8]     (~30 min on 8 cores)
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

OUT = os.path.join(ROOT, "tests", "golden", "full_width_digests.npz")
BOARDS = 65536
PLIES = 2000
# (name, seed, opponent, agent colour)
CASES = (("none", 779001, 0, "WHITE"), ("random_white", 779002, 1, "WHITE"), ("random_black", 779003, 1, "BLACK"))


def main():
    import oracle as O

    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 1)
    a = ap.parse_args()
    O.build()
    out = {"boards": np.int64(BOARDS), "plies": np.int64(PLIES)}
    for name, seed, opp, color in CASES:
        t0 = time.time()
        out[f"{name}_digest"] = O.rollout_digests(seed, BOARDS, PLIES, opponent=opp, agent_white=color == "WHITE",
                                                  threads=a.threads)
        out[f"{name}_seed"] = np.int64(seed)
        print(f"{name}: {BOARDS} boards x {PLIES} plies, {time.time() - t0:.0f} s", flush=True)
    np.savez(OUT, **out)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
