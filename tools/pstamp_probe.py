"""Diagnostic only: where a fused ply's time goes, per role -- the cycles of each segment of
k_env_rollout2<false, 0> (phase work and barrier waits, s_memtime), summed over a launch of
--plies plies and averaged per ply over the waves (build: tools/build_variants.sh pst
"-DGC_PSTAMPS" -> tools/_lib_pst.so).  Segments: phase 0 | wait A | phase 1 | wait B |
phase 2 | wait C | phase 3 (outcome, pick / commit) | wait D (next action to W1)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
L = ctypes.CDLL(os.environ.get("PST_LIB") or os.path.join(ROOT, "tools", "_lib_pst.so"))
P = ctypes.c_void_p
L.gc_env_create.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_uint64, P, P]
L.gc_env_rollout.argtypes = [P, ctypes.c_int, P, P, P, P, P]
L.gc_debug_pstamps.argtypes = [P, ctypes.c_int, P]
n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
plies = int(sys.argv[2]) if len(sys.argv) > 2 else 200
pmap = int(os.environ.get("PST_MAP", "2"))
h = P()
assert L.gc_env_create(0, n, 0x5EED + 3, None, ctypes.byref(h)) == 0
assert L.gc_env_rollout(h, 1000, None, None, None, None, None) == 0  # steady state
quad = os.environ.get("PST_QUAD") == "1"  # the quad kernel (k_env_rollout4): 4 waves per 64 boards
waves = ((n + 127) // 128) * (8 if quad else 4)
out = np.zeros(waves * 12, dtype=np.uint64)
assert L.gc_debug_pstamps(h, plies, out.ctypes.data_as(P)) == 0
raw = out.reshape(-1, 12)
st = raw[:, :8].astype(np.float64) / plies
where = (raw[:, 8] >> np.uint64(44)).astype(np.int64)  # placement: cu | sh | se | simd | xcc
hi = ~np.uint64((1 << 44) - 1)
raw[:, 8] = (raw[:, 8] & np.uint64((1 << 44) - 1)) | (raw[:, 9] & hi)  # the clock's own top bits back
rt = raw[:, 8:].astype(np.int64)  # 100 MHz: wave start, entry loads done, first ply done, last ply done
t0 = rt[:, 0].min()
us = (rt - t0) / 100.0
print(f"launch anatomy ({plies} plies, us from the first wave's start): last wave start {us[:, 0].max():.2f}; "
      f"entry loads mean {(us[:, 1] - us[:, 0]).mean():.2f}; first ply mean {(us[:, 2] - us[:, 1]).mean():.2f}, "
      f"later plies mean {((us[:, 3] - us[:, 2]) / max(plies - 1, 1)).mean():.3f}; wave end mean {us[:, 3].mean():.2f}, "
      f"p90 {np.percentile(us[:, 3], 90):.2f}, max {us[:, 3].max():.2f}")
if quad:  # k_env_rollout4: 8 waves per workgroup, roles (w & 3) ^ 2 * quad
    w = np.arange(waves) % 8
    role = (w & 3) ^ (((w >> 2) & 1) << 1)
    if os.environ.get("PST_WG") == "1":  # one quad per workgroup (QUADS_WG=1): roles 0-3 in order
        role = w & 3
    names = ["phase 0", "wait A", "phase 1", "wait B", "phase 2", "wait C", "phase 3", "wait D"]
    roles = (0, 1, 2, 3)
else:
    w = np.arange(waves) % 4
    role = np.where(pmap == 2, (w ^ (w >> 1)) & 1, w & 1)
    names = ["phase 0", "wait A", "phase 1", "wait B", "phase 2", "wait C", "phase 3", "wait D"]
    roles = (0, 1)
for r in roles:
    s = st[role == r]
    tot = s.sum(axis=1).mean()
    print(f"[{'Q' if quad else 'W'}{r}] {len(s)} waves, {tot:.0f} cycles per ply")
    for k in range(len(names)):
        print(f"   {names[k]:>8}: {s[:, k].mean():7.0f}  ({s[:, k].mean() / tot:5.1%})")
if quad:  # where the slow waves run (k_env_rollout4): wave end and per-ply time by XCD and by CU
    xcc = where >> 9
    cu_key = where & 0x7F | (xcc << 7)
    end = us[:, 3]
    per = (us[:, 3] - us[:, 2]) / max(plies - 1, 1)
    print("wave end by XCD (mean / max us):", " ".join(f"{x}:{end[xcc == x].mean():.1f}/{end[xcc == x].max():.1f}"
                                                        for x in np.unique(xcc)))
    print("per-ply us by XCD (mean / max):", " ".join(f"{x}:{per[xcc == x].mean():.3f}/{per[xcc == x].max():.3f}"
                                                       for x in np.unique(xcc)))
    _, cu_inv, cu_cnt = np.unique(cu_key, return_inverse=True, return_counts=True)
    print(f"CUs used {len(cu_cnt)}, waves per CU: " + ", ".join(f"{c}x{k}" for c, k in zip(*np.unique(cu_cnt, return_counts=True))))
    print("end percentiles (us):", " ".join(f"p{q}:{np.percentile(end, q):.1f}" for q in (0, 10, 25, 50, 75, 90, 99, 100)))
    wg = np.arange(waves) // 8
    wg_end = np.array([end[wg == g].max() for g in range(wg.max() + 1)])
    wg_per = np.array([per[wg == g].mean() for g in range(wg.max() + 1)])
    print("workgroup end percentiles (us):", " ".join(f"p{q}:{np.percentile(wg_end, q):.1f}" for q in (0, 10, 50, 90, 100)))
    # per CU: the mean per-ply time of its waves; the spread across CUs says whether the tail is
    # the place (a slow CU / XCD) or the boards (a workgroup's own work)
    cu_per = np.array([per[cu_inv == c].mean() for c in range(len(cu_cnt))])
    print("per-ply us by CU: " + " ".join(f"p{q}:{np.percentile(cu_per, q):.3f}" for q in (0, 10, 50, 90, 100)))
    # the two workgroups of a CU: how alike their per-ply times are (same place, different boards)
    pairs = {}
    for g in range(wg.max() + 1):
        pairs.setdefault(int(cu_key[wg == g][0]), []).append(g)
    d = [abs(wg_per[a[0]] - wg_per[a[1]]) for a in pairs.values() if len(a) == 2]
    print(f"CUs with two workgroups: {len(d)}; |per-ply difference| mean {np.mean(d):.3f} us, max {np.max(d):.3f}")
    # which of a CU's two workgroups is the slow one: the later-dispatched (higher index, later
    # start)?  and the SIMDs its waves sit on
    first = np.array([us[wg == g, 0].min() for g in range(wg.max() + 1)])
    slow_later = slow_higher = 0
    for a in pairs.values():
        if len(a) != 2:
            continue
        f, sl = (a[0], a[1]) if wg_per[a[0]] <= wg_per[a[1]] else (a[1], a[0])
        slow_later += first[sl] > first[f]
        slow_higher += sl > f
    nwg = wg.max() + 1
    print(f"slow workgroup of a CU: started later in {slow_later} of {len(pairs)}, higher index in {slow_higher}; "
          f"per-ply us by index half: {wg_per[:nwg // 2].mean():.3f} / {wg_per[nwg // 2:].mean():.3f}")
    simd = (where >> 7) & 3
    for g in list(pairs.values())[:3]:
        print("  CU sample:", [(int(x), f"{wg_per[x]:.3f}", f"start {first[x]:.2f}",
                               "simds " + "".join(str(int(v)) for v in simd[wg == x])) for x in g])
    sys.exit(0)

# where the slow waves run: wave end by XCD, by CU load and by SIMD load
xcc = where >> 9
cu_key = where & 0x7F | (xcc << 7)        # cu, sh, se within the XCD
simd_key = where | 0
end = us[:, 3]
print("wave end by XCD (mean / max us):", " ".join(f"{x}:{end[xcc == x].mean():.1f}/{end[xcc == x].max():.1f}"
                                                    for x in np.unique(xcc)))
_, cu_inv, cu_cnt = np.unique(cu_key, return_inverse=True, return_counts=True)
_, si_inv, si_cnt = np.unique(simd_key, return_inverse=True, return_counts=True)
print(f"CUs used {len(cu_cnt)}, waves per CU: " + ", ".join(f"{c}x{n}" for c, n in zip(*np.unique(cu_cnt, return_counts=True))))
print(f"SIMDs used {len(si_cnt)}, waves per SIMD: " + ", ".join(f"{c}x{n}" for c, n in zip(*np.unique(si_cnt, return_counts=True))))
wl = si_cnt[si_inv]
for c in np.unique(wl):
    print(f"  waves on a SIMD with {c} waves: end mean {end[wl == c].mean():.1f} max {end[wl == c].max():.1f} "
          f"per-ply {((us[:, 3] - us[:, 2]) / max(plies - 1, 1))[wl == c].mean():.3f}")
blk = np.arange(waves) // 4
print("wave end by block % 8:", " ".join(f"{b}:{end[blk % 8 == b].mean():.1f}" for b in range(8)))
print("end percentiles (us):", " ".join(f"p{q}:{np.percentile(end, q):.1f}" for q in (0, 10, 25, 50, 75, 90, 99, 100)))

# the two workgroups sharing a CU: the one dispatched first (lower block index) against the other
cu_ids = np.unique(cu_key)
d_first, first_wins = [], 0
for c in cu_ids:
    m = np.nonzero(cu_key == c)[0]
    bl = np.unique(blk[m])
    if len(bl) != 2:
        continue
    e0, e1 = end[m[blk[m] == bl[0]]].mean(), end[m[blk[m] == bl[1]]].mean()
    d_first.append(e1 - e0)
    first_wins += e0 < e1
d_first = np.array(d_first)
print(f"CUs with two workgroups: {len(d_first)}; lower block index finishes first on {first_wins}; "
      f"end(later WG) - end(earlier WG): mean {d_first.mean():.1f} us, |mean| {np.abs(d_first).mean():.1f}, "
      f"block distance of the pair: {sorted(set(int(np.diff(np.unique(blk[cu_key == c]))[0]) for c in cu_ids[:64] if len(np.unique(blk[cu_key == c])) == 2))[:8]}")
