"""Diagnostic: restore into a pre-stepped env vs the uninterrupted env, first divergence."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-chess_amd"))
from gym_chess_amd.env import BatchedChessEnv  # noqa: E402

n, seed, cut = 256, 4711, 150
a = BatchedChessEnv(n, device=0, seed=seed)
a.step_random(cut)
blob = a.checkpoint()
f = BatchedChessEnv(n, device=0, seed=seed)
f.step_random(int(sys.argv[1]) if len(sys.argv) > 1 else 37)
f.load(blob)
blob2 = f.checkpoint()
hdr = 8 + 4 * 6 + 8 + 56 + 8
print("blob sizes", len(blob), len(blob2))
sa = np.frombuffer(blob, np.uint8)[hdr:hdr + 80 * n]
sb = np.frombuffer(blob2, np.uint8)[hdr:hdr + 80 * n]
diff = np.nonzero(sa != sb)[0]
print("slab bytes differing:", len(diff), "offsets/n:", sorted(set((diff // n).tolist()))[:20])
ea = np.frombuffer(blob, np.uint64)[(hdr + 80 * n) // 8:].reshape(-1, 8)
eb = np.frombuffer(blob2, np.uint64)[(hdr + 80 * n) // 8:].reshape(-1, 8)
print("entries", ea.shape, eb.shape)
sa_set = {tuple(r) for r in ea}
sb_set = {tuple(r) for r in eb}
print("entry sets equal:", sa_set == sb_set)
for p in range(300):
    a.step_random(1)
    f.step_random(1)
    oa, of = a.outputs(), f.outputs()
    bad = [i for i in range(n) if any(oa[k][i] != of[k][i] for k in oa)]
    ba, ma = a.boards()
    bf, mf = f.boards()
    badb = np.nonzero((ba != bf).any(axis=1) | (ma != mf).any(axis=1))[0]
    if bad or len(badb):
        i = bad[0] if bad else int(badb[0])
        print("ply", p, "boards", bad[:10], badb[:10])
        print({k: (int(oa[k][i]), int(of[k][i])) for k in oa})
        print("meta", ma[i], mf[i])
        break
else:
    print("no divergence in 300 plies")
