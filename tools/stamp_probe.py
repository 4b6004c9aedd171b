"""Diagnostic only: per-phase wave time of k_env_step<true> from s_memtime stamps
(build: hipcc ... -DGC_STAMPS -o tools/_build_stamps.so gym-chess_amd/csrc/gymchess.hip).
Phases: 0 entry | 1 inputs loaded | 2 probe issued | 3 apply+gen_init+check | 4 gen_moves |
5 repetition commit | 6 reset/regen | 7 pick.  Shares, not absolute times (stamps serialise)."""
import ctypes
import os
import sys

import numpy as np

L = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "_build_stamps.so"))
P = ctypes.c_void_p
L.gc_env_create.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_uint64, P, P]
L.gc_env_step_random.argtypes = [P, ctypes.c_int]
L.gc_debug_stamps.argtypes = [P, ctypes.c_int, P]
L.gc_env_synchronize.argtypes = [P]
n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
h = P()
assert L.gc_env_create(0, n, 0x5EED + 3, None, ctypes.byref(h)) == 0
assert L.gc_env_step_random(h, 400) == 0
L.gc_env_synchronize(h)
out = np.zeros(((n + 63) // 64) * 8, dtype=np.uint64)
assert L.gc_debug_stamps(h, 1, out.ctypes.data_as(P)) == 0
st = out.reshape(-1, 8).astype(np.int64)
base = st[:, 0]
names = ["load inputs", "probe issue", "apply+gen_init+chk", "gen_moves", "rep commit", "reset/regen", "pick"]
tot = (st[:, 7] - st[:, 0]).astype(float)
print(f"waves {len(st)}  mean wave span {tot.mean():.0f} ticks  (s_memtime units)")
for k in range(1, 8):
    d = (st[:, k] - st[:, k - 1]).astype(float)
    ok = (st[:, k] >= st[:, k - 1]) & (st[:, k - 1] > 0)
    q = np.percentile(d[ok], [50, 75, 90, 99]) if ok.any() else [0, 0, 0, 0]
    print(f"{names[k-1]:>22}: mean {d[ok].mean():8.0f}  p50/75/90/99 {q[0]:7.0f} {q[1]:7.0f} {q[2]:7.0f} {q[3]:7.0f}  "
          f"share {d[ok].sum()/tot[ok].sum():5.1%}  (waves {ok.sum()})")
start = st[:, 0] - st[:, 0].min()
print("wave start spread (ticks): p50 %d p99 %d max %d" % (np.median(start), np.percentile(start, 99), start.max()))
end = st[:, 7] - st[:, 0].min()
print("wave end   spread (ticks): p50 %d p99 %d max %d" % (np.median(end), np.percentile(end, 99), end.max()))
