"""Diagnostic only: wave start ramp and end spread of one k_env_step2 launch, in microseconds.
Needs the real-time stamp build:
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -mllvm -amdgpu-kernarg-preload-count=16 \
        -DGC_STAMPS -DGC_STAMPS_REAL -o tools/_build_stamps_rt.so gym-chess_amd/csrc/gymchess.hip
(every stamp is s_memrealtime, 100 MHz, one clock for all CUs)."""
import ctypes
import os
import time

import numpy as np

L = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "_build_stamps_rt.so"))
P = ctypes.c_void_p
L.gc_env_create.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_uint64, P, P]
L.gc_env_step_random.argtypes = [P, ctypes.c_int]
L.gc_debug_stamps.argtypes = [P, ctypes.c_int, P]
L.gc_env_synchronize.argtypes = [P]
L.gc_env_record_event.argtypes = [P, ctypes.c_int]
L.gc_env_elapsed_ms.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_float)]
for n in (16384, 65536, 131072):
    h = P()
    assert L.gc_env_create(0, n, 0x5EED + 3, None, ctypes.byref(h)) == 0
    assert L.gc_env_step_random(h, 400) == 0
    L.gc_env_synchronize(h)
    L.gc_env_record_event(h, 0)
    assert L.gc_env_step_random(h, 200) == 0
    L.gc_env_record_event(h, 1)
    L.gc_env_synchronize(h)
    ms = ctypes.c_float()
    L.gc_env_elapsed_ms(h, 0, 1, ctypes.byref(ms))
    out = np.zeros(((n + 63) // 64) * 16, dtype=np.uint64)
    assert L.gc_debug_stamps(h, 1, out.ctypes.data_as(P)) == 0
    st = out.reshape(-1, 8).astype(np.int64)
    r0, r1 = st[:, 0], st[:, 7]
    b = r0.min()
    us = lambda x: x / 100.0  # noqa: E731
    print(f"n={n}: waves {len(st)}  per launch {ms.value * 1000 / 200:.2f} us (events)  "
          f"start ramp p50/p90/max {us(np.percentile(r0 - b, 50)):.2f}/{us(np.percentile(r0 - b, 90)):.2f}/{us((r0 - b).max()):.2f}  "
          f"span mean {us(np.mean(r1 - r0)):.2f}  first start -> last end {us(r1.max() - b):.2f}  "
          f"end p10/p50/max {us(np.percentile(r1 - b, 10)):.2f}/{us(np.percentile(r1 - b, 50)):.2f}/{us((r1 - b).max()):.2f}")
