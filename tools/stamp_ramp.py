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
    raw = out.reshape(-1, 8)
    where = (raw[:, 0] >> np.uint64(44)).astype(np.int64)  # cu | sh<<4 | se<<5 | simd<<7 | xcc<<9
    lowm = np.uint64((1 << 44) - 1)
    raw[:, 0] = (raw[:, 0] & lowm) | (raw[:, 1] & ~lowm)  # high clock bits from the next stamp
    st = raw.astype(np.int64)
    r0, r1 = st[:, 0], st[:, 7]
    b = r0.min()
    us = lambda x: x / 100.0  # noqa: E731
    print(f"n={n}: waves {len(st)}  per launch {ms.value * 1000 / 200:.2f} us (events)  "
          f"start ramp p50/p90/max {us(np.percentile(r0 - b, 50)):.2f}/{us(np.percentile(r0 - b, 90)):.2f}/{us((r0 - b).max()):.2f}  "
          f"span mean {us(np.mean(r1 - r0)):.2f}  first start -> last end {us(r1.max() - b):.2f}  "
          f"end p10/p50/max {us(np.percentile(r1 - b, 10)):.2f}/{us(np.percentile(r1 - b, 50)):.2f}/{us((r1 - b).max()):.2f}")
    # the tail: which waves end last, and why (start late? long span? which phase?)
    end = r1 - b
    slow = end >= np.percentile(end, 95)
    names = ["load", "ph0+1", "bar1", "ph2", "bar2", "out/pick", "stores"]
    ph = np.diff(st, axis=1) / 100.0
    print(f"   last 5% of waves to end: start mean {us(np.mean(r0[slow]-b)):.2f} (all {us(np.mean(r0-b)):.2f}) "
          f"span mean {us(np.mean(r1[slow]-r0[slow])):.2f} (all {us(np.mean(r1-r0)):.2f})")
    print("   phases (us) slow / all: " + "  ".join(f"{nm} {ph[slow, k].mean():.2f}/{ph[:, k].mean():.2f}" for k, nm in enumerate(names)))
    if len(st) == 2 * ((n + 63) // 64):
        w = np.arange(len(st))
        print(f"   slow waves W0/W1: {int(slow[w % 2 == 0].sum())}/{int(slow[w % 2 == 1].sum())}; "
              f"slow block ids (first 16): {sorted((w[slow] // 2).tolist())[:16]}")
    cu = where & 0x7F | ((where >> 9) << 7)  # cu, sh, se, xcc
    simd = (where >> 7) & 3
    ucu, ccu = np.unique(cu, return_counts=True)
    key = cu * 4 + simd
    uk, ck = np.unique(key, return_counts=True)
    per_simd = dict(zip(uk.tolist(), ck.tolist()))
    wsimd = np.array([per_simd[k] for k in key.tolist()])
    print(f"   CUs used {len(ucu)}; waves per CU min/max {ccu.min()}/{ccu.max()}; waves per SIMD hist "
          f"{dict(zip(*np.unique(ck, return_counts=True)))}")
    print(f"   slow waves: their SIMD's wave count mean {wsimd[slow].mean():.2f} (all {wsimd.mean():.2f}); "
          f"span by SIMD load: " + "  ".join(f"{v}: {np.mean((r1-r0)[wsimd == v])/100:.2f}us" for v in sorted(set(wsimd.tolist()))))
