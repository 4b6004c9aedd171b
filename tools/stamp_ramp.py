"""Diagnostic only (temporary layout: slot 2/3 = s_memrealtime at wave start/end, 100 MHz):
wave start ramp and end spread of one k_env_step2 launch, in microseconds."""
import ctypes, os
import numpy as np
L = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "_build_stamps.so"))
P = ctypes.c_void_p
L.gc_env_create.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_uint64, P, P]
L.gc_env_step_random.argtypes = [P, ctypes.c_int]
L.gc_debug_stamps.argtypes = [P, ctypes.c_int, P]
L.gc_env_synchronize.argtypes = [P]
for n in (16384, 65536):
    h = P()
    assert L.gc_env_create(0, n, 0x5EED + 3, None, ctypes.byref(h)) == 0
    assert L.gc_env_step_random(h, 400) == 0
    L.gc_env_synchronize(h)
    out = np.zeros((n // 64) * 16, dtype=np.uint64)
    assert L.gc_debug_stamps(h, 1, out.ctypes.data_as(P)) == 0
    st = out.reshape(-1, 8).astype(np.int64)
    r0, r1 = st[:, 2], st[:, 3]
    b = r0.min()
    us = lambda x: x / 100.0  # noqa: E731
    print(f"n={n}: waves {len(st)}  start ramp p50/p90/max {us(np.percentile(r0-b,50)):.2f}/{us(np.percentile(r0-b,90)):.2f}/"
          f"{us((r0-b).max()):.2f} us   span mean {us(np.mean(r1-r0)):.2f} us ({np.mean(st[:,7]-st[:,0]):.0f} ticks)   "
          f"first start -> last end {us(r1.max()-b):.2f} us   end p50/max {us(np.percentile(r1-b,50)):.2f}/{us((r1-b).max()):.2f}")
