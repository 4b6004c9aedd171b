"""Diagnostic only (temporary layout: stamp slot 3 = XCC id): per-XCD wave start / end
spread of one k_env_step2 launch vs the mean wave span."""
import ctypes, os
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
out = np.zeros((n // 64) * 16, dtype=np.uint64)
assert L.gc_debug_stamps(h, 1, out.ctypes.data_as(P)) == 0
st = out.reshape(-1, 8).astype(np.int64)
xcc = st[:, 3]
for x in sorted(set(xcc.tolist()))[:8]:
    s = st[xcc == x]
    t0, t7 = s[:, 0], s[:, 7]
    print(f"xcc {x}: waves {len(s)}  start spread {t0.max()-t0.min():6d}  end spread {t7.max()-t7.min():6d}  "
          f"first start -> last end {t7.max()-t0.min():6d}  mean span {np.mean(t7-t0):7.0f}  "
          f"start p50/p90 {np.percentile(t0-t0.min(),50):5.0f}/{np.percentile(t0-t0.min(),90):5.0f}")
