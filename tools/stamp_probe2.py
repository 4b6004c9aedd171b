"""Diagnostic only: per-phase wave time of the paired step kernel k_env_step2 from s_memtime
stamps (build: hipcc ... -DGC_STAMPS -o tools/_build_stamps.so gym-chess_amd/csrc/gymchess.hip).
Stamps: 0 entry | 1 inputs loaded | 2 phase-1 work | 3 barrier 1 | 4 phase-2 work |
5 barrier 2 | 6 outcome + pick (W0) / outcome (W1) | 7 stores issued.  GC_STEP1=1 probes
the one-wave kernel instead (tools/stamp_probe.py phases)."""
import ctypes
import os
import sys

import numpy as np

L = ctypes.CDLL(os.environ.get("STAMP_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "_build_stamps.so"))
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
out = np.zeros(((n + 63) // 64) * 16, dtype=np.uint64)
assert L.gc_debug_stamps(h, 1, out.ctypes.data_as(P)) == 0
st = out.reshape(-1, 8).astype(np.int64)
if os.environ.get("GC_STEP1"):
    st = st[: (n + 63) // 64]
    roles = {"one wave": st}
else:
    roles = {"W0": st[0::2], "W1": st[1::2]}
names = ["load inputs", "phase-1 work", "barrier 1", "phase-2 work", "barrier 2", "outcome/pick", "stores"]
for rn, s in roles.items():
    tot = (s[:, 7] - s[:, 0]).astype(float)
    print(f"[{rn}] waves {len(s)}  mean wave span {tot.mean():.0f} ticks")
    for k in range(1, 8):
        d = (s[:, k] - s[:, k - 1]).astype(float)
        ok = (s[:, k] >= s[:, k - 1]) & (s[:, k - 1] > 0)
        q = np.percentile(d[ok], [50, 90, 99]) if ok.any() else [0, 0, 0]
        print(f"  {names[k-1]:>14}: mean {d[ok].mean():7.0f}  p50/90/99 {q[0]:7.0f} {q[1]:7.0f} {q[2]:7.0f}  "
              f"share {d[ok].sum()/tot[ok].sum():5.1%}")
