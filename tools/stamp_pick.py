"""Diagnostic only (temporary stamp layout): W0 phase-3 split.  Stamps: 0 entry | 1 loaded |
4 phase-2 end | 5 barrier 2 | 2 outcome done | 3 before select_action (non-table lanes) |
6 pick done | 7 end."""
import ctypes, os, sys
import numpy as np
L = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "_build_stamps.so"))
P = ctypes.c_void_p
L.gc_env_create.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_uint64, P, P]
L.gc_env_step_random.argtypes = [P, ctypes.c_int]
L.gc_debug_stamps.argtypes = [P, ctypes.c_int, P]
L.gc_env_synchronize.argtypes = [P]
n = 65536
h = P()
assert L.gc_env_create(0, n, 0x5EED + 3, None, ctypes.byref(h)) == 0
assert L.gc_env_step_random(h, 400) == 0
L.gc_env_synchronize(h)
out = np.zeros(((n + 63) // 64) * 16, dtype=np.uint64)
assert L.gc_debug_stamps(h, 1, out.ctypes.data_as(P)) == 0
st = out.reshape(-1, 8).astype(np.int64)[0::2]
for a, b, name in ((5, 2, "outcome"), (2, 3, "to select"), (3, 6, "select_action"), (2, 6, "whole pick"), (6, 7, "stores")):
    d = (st[:, b] - st[:, a]).astype(float)
    ok = (st[:, b] > 0) & (st[:, a] > 0) & (d >= 0)
    print(f"{name:>14}: mean {d[ok].mean():7.0f} p50 {np.median(d[ok]):7.0f} (waves {ok.sum()})")
