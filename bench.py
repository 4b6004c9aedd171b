#!/usr/bin/env python3
"""Benchmark: env.step() throughput of the batched chess env on MI355X.

Workload (BASELINE.json configs[2], the config the metric is quoted on): 65 536 boards per
GPU, random-policy self-play to terminal with auto-reset -- the reference's benchmark
driver (/root/reference/gym_chess/test/v2/test_benchmark.py:9-43) vectorised.  One "step"
= one env.step() on every board: the policy's action through the full chess_v2.py step
bookkeeping (next_state, update_state, 3-fold on the pre-move board, move cap, mate bonus),
the next side's legal move set, the Philox pick of the next action, reset of finished
boards, and the step's outputs (action played, reward, done, reason) of every board written
to a per-ply trace in HBM.  The K timed steps are ONE launch of the fused rollout kernel
k_env_rollout4 (four waves per 64 boards; gc_env_rollout_device: the state stays in registers between plies; every
ply's window probe / commit and outputs go through HBM).  State, repetition windows and
outputs stay in HBM; nothing crosses PCIe in the timed region.  The launched form (one
kernel launch per ply, k_env_step2 over two board-range streams) is timed beside it as
"launched_step".

The batch is first settled into steady state (a fused rollout of --settle plies, then
--warmup steps), so the timed steps see mid/late-game boards, resets and terminals in their
steady-state proportions, whatever --warmup is.

  python bench.py [--gpus N --steps K --warmup W --boards B]
      N replicas in ONE process: one host thread + one env handle per device (no torch)
  python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
      one process per GPU; barrier / max / sum through a file group (gym_chess_amd.replicas)
  (boards sharded, no data-path collective: "scaling": "weak")

Prints ONE JSON line (rank 0).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gym-chess_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip-level parameters (8.0 TB/s spec)

# algorithmic bytes per board per fused rollout ply (BASELINE.md CPU-baseline
# plan): state read 80 + state write 80 + repetition history 8h + action 8 + outputs 5
# = 173 + 8h B, h = the mean repetition-window length (boards since the last pawn move or
# capture) measured over the timed steps
def alg_bytes_fused(h):
    return 173.0 + 8.0 * h


# the fused rollout's kernel by waves per 64 boards (gc_env_rollout_waves)
ROLLOUT_KERNEL = {4: "k_env_rollout4", 2: "k_env_rollout2<false, 0>", 1: "k_env_rollout<false>"}


# the launched step k_env_step2 (one kernel per ply; DESIGN.md §5 byte model):
#   state 7x8 B bitboards + 4 B meta, read + write                     120
#   action read + next-action write (u16)                                4
#   Philox draw counter, step counter, window generation: read + write  24
#   outputs reward i32 + done u8 + reason u8                              6
#   3-fold window: one 64-B table probe read                             64
#   3-fold window: 64-B entry write (reversible plies; counted always)   64
ALG_BYTES_PER_BOARD = 120 + 4 + 24 + 6 + 64 + 64

# the PMC profiles the traffic / VALU figures come from (rocprofv3 passes, tools/gpu_run.sh
# pmc*; tools/pmc_summary.py); counters cannot be read from inside this process
PMC_FILE = os.path.join(ROOT, "profiles", "pmc_rollout_latest.json")  # the driver's K = 20 launch
PMC_FILE_LONG = os.path.join(ROOT, "profiles", "pmc_rollout_long_latest.json")  # a K = 1 000 launch
PMC_STEP_FILE = os.path.join(ROOT, "profiles", "pmc_traffic_latest.json")


def load_pmc(path):
    if not os.path.exists(path):
        return None
    try:
        return json.load(open(path))
    except (OSError, ValueError):
        return None


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None, help="replicas (GPUs); default 1, or WORLD_SIZE under a launcher")
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--settle", type=int, default=1000,
                    help="fused-rollout plies before --warmup: moves the batch from all-startpos into steady state")
    ap.add_argument("--boards", type=int, default=65536)
    ap.add_argument("--seed", type=int, default=0x5EED + 3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-boards", type=int, default=32768)
    ap.add_argument("--cpu-sample-plies", type=int, default=300)
    ap.add_argument("--cpu1-sample-boards", type=int, default=4096, help="boards of the single-core CPU sample")
    ap.add_argument("--launched-steps", type=int, default=300,
                    help="also time the launched step (one k_env_step2 launch per ply, 0 = skip)")
    ap.add_argument("--perft-roots", type=int, default=65536, help="perft leg on mid-game FEN roots (0 = skip)")
    ap.add_argument("--variant-steps", type=int, default=300,
                    help="also time step() with opponent='random' and with rules='fide' (SURVEY 8f rows 2, 4; 0 = skip)")
    ap.add_argument("--api-steps", type=int, default=300,
                    help="also time the API-shaped step on device buffers (mask + obs out; 0 = skip)")
    ap.add_argument("--single-episodes", type=int, default=10,
                    help="configs[0]: the reference benchmark driver on the single-board env (0 = skip)")
    ap.add_argument("--concurrent-ms", type=float, default=0.0,
                    help="replicas' common-interval leg (>= this many ms per replica); always on (250 ms) for N > 1")
    ap.add_argument("--configs1-roots", type=int, default=4096,
                    help="configs[1]: start-position roots of the perft(3) leg (0 = skip)")
    ap.add_argument("--perft-depth", type=int, default=5)
    ap.add_argument("--perft-subsample", type=int, default=256,
                    help="roots of the fixed strided subsample checked (and CPU-timed) one ply shallower")
    ap.add_argument("--oracle-perft-roots", type=int, default=8,
                    help="roots of the perft leg checked against the oracle at --perft-depth (also its CPU baseline)")
    return ap.parse_args()


def cpu_baseline(args):
    """Oracle (C restatement of lib.rs + chess_v2.py, test infrastructure) on the host: the
    same random self-play driver on bounded samples of boards, on all host threads (up to 16,
    the box's CPU share) and on one core (BASELINE.md CPU-baseline plan)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    threads = max(1, min(16, os.cpu_count() or 1))
    O.lib()
    t0 = time.perf_counter()
    st = O.rollout_batch(args.seed, 0, args.cpu_sample_boards, args.cpu_sample_plies, threads=threads)
    dt = time.perf_counter() - t0
    steps = int(st[0])
    t0 = time.perf_counter()
    st1 = O.rollout_batch(args.seed, 0, args.cpu1_sample_boards, args.cpu_sample_plies, threads=1)
    dt1 = time.perf_counter() - t0
    steps1 = int(st1[0])
    return {
        "value": steps / dt,
        "unit": "env_steps/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{args.cpu_sample_boards} boards x {args.cpu_sample_plies} plies random self-play "
        f"({steps} env.step calls, {dt:.1f} s) with the C oracle restating lib.rs + chess_v2.py",
        "single_core": {"value": steps1 / dt1, "unit": "env_steps/s", "cores": 1,
                        "sample": f"{args.cpu1_sample_boards} boards x {args.cpu_sample_plies} plies "
                                  f"({steps1} env.step calls, {dt1:.1f} s)"},
    }


def midgame_fens(n, seed, device):
    """configs[3]: n mixed mid-game positions as FEN strings.  Board i is taken after
    10 + (i*7919 mod 31) plies of seeded uniform-random self-play from the start position
    (SURVEY.md §8d config 4), exported through the C-ABI's FEN codec."""
    import numpy as np

    from gym_chess_amd.env import BatchedChessEnv
    from gym_chess_amd.fen import arrays_to_fen

    src = BatchedChessEnv(n, device=device, seed=seed)
    ply = 10 + (np.arange(n, dtype=np.int64) * 7919) % 31
    b = np.zeros((n, 64), np.int8)
    m = np.zeros((n, 8), np.uint8)
    src.step_random(10)
    for p in range(10, 41):
        if p > 10:
            src.step_random(1)
        sel = ply == p
        bb, mm = src.boards()
        b[sel], m[sel] = bb[sel], mm[sel]
    src.close()
    return [arrays_to_fen(b[i], m[i]) for i in range(n)]


def perft_leg(args, rep):
    """configs[3]: mid-game FEN roots, perft(depth) through the engine C-ABI (device level
    expansion, then the split leaf pass: depth-3 subtrees split to sorted depth-2 ones).  The
    first --oracle-perft-roots roots of replica 0 are recomputed by the oracle at the same
    depth and must match exactly; at N=1 that run is also the perft CPU baseline."""
    import numpy as np

    from gym_chess_amd.engine import Engine, perft_dedup_stats, perft_leaf_stats, perft_path_counts
    from gym_chess_amd.fen import fen_to_arrays

    def prep(rp):
        fens = midgame_fens(args.perft_roots, rp.board_seed(0x5EED + 4), rp.device)
        arr = [fen_to_arrays(f) for f in fens]
        b = np.stack([a[0] for a in arr])
        m = np.stack([a[1] for a in arr])
        eng = Engine(rp.device)
        b, m = eng.update_state(b, m)  # FEN carries no check flags: update_state, as chess_v2.py:204 does
        eng.perft(b[:256], m[:256], 2)  # load the perft kernels outside the timed region
        return eng, b, m

    ctx = rep.run(prep)
    paths0 = perft_path_counts()
    leaf0 = perft_leaf_stats()
    dd0 = perft_dedup_stats()

    def run(rp):
        eng, b, m = ctx[rep.local.index(rp)]
        t0 = time.perf_counter()
        nodes = eng.perft(b, m, args.perft_depth)
        return nodes, time.perf_counter() - t0

    res, dtm = rep.timed(run)
    paths1 = perft_path_counts()
    leaf1 = perft_leaf_stats()
    dd1 = perft_dedup_stats()
    for eng, _, _ in ctx:
        eng.close()
    tot = rep.sum(float(sum(float(r.sum()) for r in res)))
    b, m = ctx[0][1], ctx[0][2]
    castle = int((m[:, 1:5] != 0).any(axis=1).sum())
    prom = int(((b[:, 8:16] == 6) | (b[:, 48:56] == -6)).any(axis=1).sum())
    check = int((m[:, 5:7] != 0).any(axis=1).sum())
    out = {"value": tot / dtm, "unit": "perft_nodes/s", "roots_per_gpu": args.perft_roots, "depth": args.perft_depth,
           "nodes": tot, "seconds": dtm,
           "leaf_pass": {k: paths1[k] - paths0[k] for k in paths0},
           "roots_with": {"castle_right": castle, "pawn_on_7th": prom, "side_in_check": check}}
    # the leaf kernel (k_perft2_val: one lane = one distinct depth-2 subtree, read in order,
    # last ply bulk-counted): where the time goes.  It is VALU-bound -- 72 algorithmic HBM bytes
    # per subtree (the 64-B root record in, its count added into the parent's sum) against ~1e3
    # leaves -- so its roof is the VALU issue rate (PMC profile, tools/gpu_run.sh pmcp*).
    # Transpositions (round 4): the split pass counts one depth-2 subtree per distinct position
    # of a chunk (exact: whole-record compare) and adds that count to every parent the position
    # occurs under -- since round 5 the records sorted by hash tag, each leader's leaf lane
    # adding its count into its followers' parents.  GC_PERFT_DEDUP=0 counts every record
    # (k_perft2_rec, 72 B).
    dedup = os.environ.get("GC_PERFT_DEDUP", "1") != "0"
    alg_sub = 72
    la, sub, kms = (b - a for a, b in zip(leaf0, leaf1))
    recs, counted = (b - a for a, b in zip(dd0, dd1))
    if recs:
        # the leaf's own rate beside nodes/s: the transposition merge raises
        # nodes/s by counting each distinct depth-2 subtree once, not by a faster leaf
        out["transpositions"] = {"records": recs, "counted": counted, "records_per_counted": recs / max(1, counted),
                                 "merged": dedup, "records_per_s": recs / dtm, "counted_subtrees_per_s": counted / dtm}
    if la:
        kname = "k_perft2_val" if dedup else "k_perft2_rec"
        roof = {"bound": "valu", "kernel": kname, "launches": la,
                "subtrees": sub, "kernel_ms": kms, "share_of_perft_time": kms / 1e3 / len(rep.local) / dtm,
                "alg_bytes_per_subtree": alg_sub, "hbm_achieved_gbs": alg_sub * sub / (kms / 1e3) / 1e9}
        pf = os.path.join(ROOT, "profiles", "pmc_perft_latest.json")
        if os.path.exists(pf):
            try:
                pm = json.load(open(pf))
                roof["valu"] = pm.get("valu")
                roof["traffic_bytes_per_subtree"] = pm.get("hbm_bytes_per_subtree")
                roof["pmc_source"] = {"file": os.path.relpath(pf, ROOT), "profile": pm.get("profile")}
            except (OSError, ValueError):
                pass
        out["roofline"] = roof
    fx = fixture_check(args, rep, ctx[0], res[0])
    if fx is not None:
        out["fixture_check"] = fx
    k = min(args.oracle_perft_roots, args.perft_roots)
    if rep.rank == 0 and k > 0:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O

        threads = max(1, min(16, os.cpu_count() or 1))
        # roots spread over the whole batch: the first, the last and evenly strided ones
        idx = np.unique(np.linspace(0, args.perft_roots - 1, k).round().astype(np.int64))
        t0 = time.perf_counter()
        cn = O.perft_by_children(b[idx], m[idx], args.perft_depth, threads=threads)
        cdt = time.perf_counter() - t0
        mism = idx[np.nonzero(cn != res[0][idx])[0]]
        assert len(mism) == 0, f"oracle perft({args.perft_depth}) disagrees with the device at roots {mism[:8]}"
        out["oracle_checked_roots"] = [int(x) for x in idx]
        out["oracle_checked_nodes"] = int(cn.sum())
        # BASELINE.md's fixed subsample: 256 roots strided over the batch, one ply shallower
        # (perft(5) of 256 mid-game roots is ~1e10 nodes: minutes of CPU), device vs oracle
        sub = np.arange(0, args.perft_roots, max(1, args.perft_roots // args.perft_subsample))[: args.perft_subsample]
        sd = max(1, args.perft_depth - 1)
        eng = Engine(rep.local[0].device)
        dn = eng.perft(b[sub], m[sub], sd)
        eng.close()
        t0 = time.perf_counter()
        sn = O.perft_by_children(b[sub], m[sub], sd, threads=threads)
        sdt = time.perf_counter() - t0
        bad = sub[np.nonzero(sn != dn)[0]]
        assert len(bad) == 0, f"oracle perft({sd}) disagrees with the device at roots {bad[:8]}"
        out["oracle_subsample"] = {"roots": len(sub), "stride": int(sub[1] - sub[0]) if len(sub) > 1 else 0,
                                   "depth": sd, "nodes": int(sn.sum()), "match": True}
        if rep.world_size == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = {"value": float(sn.sum()) / sdt, "unit": "perft_nodes/s", "cores": threads,
                                   "kind": "port",
                                   "sample": f"{len(sub)} roots strided over the batch x perft({sd}) "
                                   f"({int(sn.sum())} nodes, {sdt:.1f} s) with the C oracle (children handed out "
                                   f"across threads)",
                                   "spread_roots_depth5": {"value": float(cn.sum()) / cdt, "roots": len(idx),
                                                           "nodes": int(cn.sum()), "seconds": cdt}}
    return out


def perft_startpos_leg(args, rep, depth=3, reps=20):
    """configs[1]: --configs1-roots copies of the start position, perft(3) through the engine
    C-ABI (gc_engine_perft; 8 982 leaves per root under the reference rules), timed
    over `reps` calls after a warm call; every root's count must equal the oracle's.  CPU
    baseline: the oracle's perft(3) of the start position on a bounded sample of roots."""
    import numpy as np

    from gym_chess_amd import codec as C
    from gym_chess_amd.engine import Engine

    n = args.configs1_roots
    b = np.tile(np.asarray(C.DEFAULT_BOARD, np.int8).reshape(1, 64), (n, 1))
    m = np.zeros((n, 8), np.uint8)
    m[:, 0:5] = 1  # WHITE to move, all four castle rights (chess_v2.py:183-206)

    def prep(rp):
        eng = Engine(rp.device)
        eng.perft(b, m, depth)  # load the kernels
        return eng

    ctx = rep.run(prep)

    def run(rp):
        eng = ctx[rep.local.index(rp)]
        t0 = time.perf_counter()
        for _ in range(reps):
            nodes = eng.perft(b, m, depth)
        return nodes, time.perf_counter() - t0

    res, dt = rep.timed(run)
    for eng in ctx:
        eng.close()
    tot = rep.sum(float(sum(float(r.sum()) for r in res))) * reps
    out = {"value": tot / dt, "unit": "perft_nodes/s", "roots_per_gpu": n, "depth": depth, "calls": reps,
           "nodes_per_call": int(res[0].sum()), "ms_per_call": dt * 1e3 / reps,
           "form": "one gc_engine_perft call per repetition (host arrays in, per-root counts out: PCIe included)"}
    if rep.rank == 0:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O

        threads = max(1, min(16, os.cpu_count() or 1))
        t0 = time.perf_counter()
        cn = O.perft_by_children(b, m, depth, threads=threads)
        cdt = time.perf_counter() - t0
        assert (cn == cn[0]).all() and (res[0] == cn[0]).all(), "configs[1] perft differs from the oracle"
        out["oracle_nodes_per_root"] = int(cn[0])
        out["match"] = True
        if rep.world_size == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = {"value": float(cn.sum()) / cdt, "unit": "perft_nodes/s", "cores": threads,
                                   "kind": "port",
                                   "sample": f"all {n} start-position roots x perft({depth}) ({int(cn.sum())} nodes, "
                                             f"{cdt:.2f} s) with the C oracle, children handed out across threads"}
    return out


PERFT_FIXTURE = os.path.join(ROOT, "tests", "golden", "configs3_perft.npz")


def fixture_check(args, rep, ctx0, nodes):
    """configs[3] pinned at full width: rank 0's roots against the oracle's
    fixture (tests/golden/make_perft_roots.py: the same 65 536 roots regenerated by the oracle,
    every root's perft(4), every 64th root's perft(5)).  The timed run's per-root perft(5) must
    equal the fixture on its stride, and a perft(4) of every root (outside the timed region)
    must equal the fixture root by root; any difference fails the bench."""
    import numpy as np

    if rep.rank != 0 or args.perft_roots != 65536 or args.perft_depth != 5 or not os.path.exists(PERFT_FIXTURE):
        return None
    eng, b, m = ctx0
    f = np.load(PERFT_FIXTURE)
    same = bool((b == f["boards"]).all() and (m[:, :7] == f["metas"][:, :7]).all())
    assert same, "the perft roots differ from the fixture's (tests/golden/configs3_perft.npz)"
    s5 = f["stride5"]
    bad5 = s5[np.nonzero(nodes[s5] != f["perft5"])[0]]
    assert len(bad5) == 0, f"perft(5) differs from the fixture at roots {bad5[:8]}"
    from gym_chess_amd.engine import Engine

    e4 = Engine(rep.local[0].device)
    p4 = e4.perft(b, m, 4)
    e4.close()
    bad4 = np.nonzero(p4 != f["perft4"])[0]
    assert len(bad4) == 0, f"perft(4) differs from the fixture at roots {bad4[:8]}"
    return {"fixture": os.path.relpath(PERFT_FIXTURE, ROOT), "roots_equal": 65536,
            "perft4_roots_equal": 65536, "perft4_nodes": int(p4.sum()),
            "perft5_roots_equal": int(len(s5)), "perft5_stride": int(s5[1] - s5[0]),
            "perft5_stride_nodes": int(nodes[s5].sum()), "match": True}


# algorithmic bytes per board of one API-shaped step (k_env_step_api4 / _api2): state 120 r/w, action 2, draw / step counter / window generation 24 r/w, window probe 64 + entry
# write 64, outputs reward / done / reason to the caller and the env 12, the legal-action mask
# 520 (65 words), observation 64, legal count 4, the pick 2 + the env's act 2
ALG_BYTES_API = 120 + 2 + 24 + 128 + 12 + 520 + 64 + 4 + 4


def api_step_leg(args, rep, n, **env_kw):
    """The reference's call shape (chess_v2.py:219-294 + possible_actions 333-335) on device
    buffers: per step an external action per board in (here: the previous step's random-policy
    pick, so no host round trip), reward / done / reason, the int8 observation, the legal-action
    mask and count out, auto-reset of finished boards.  One launch of k_env_step_api4 (the quad
    API step; the random opponent's: k_env_step_api4_vs) per step."""
    from gym_chess_amd.env import BatchedChessEnv

    def setup(rp):
        env = BatchedChessEnv(n, device=rp.device, seed=rp.board_seed(args.seed + 11), **env_kw)
        if args.settle > 0:
            env.rollout(args.settle)
        io = env.device_io()
        for _ in range(max(args.warmup, 20)):
            env.step_device(io, autoreset=True)
        env.synchronize()
        return env, io

    ctx = rep.run(setup)

    def run(rp):
        env, io = ctx[rep.local.index(rp)]
        t0 = time.perf_counter()
        env.record_event(4)
        for _ in range(args.api_steps):
            env.step_device(io, autoreset=True)
        env.record_event(5)
        env.synchronize()
        return None, time.perf_counter() - t0

    _, dt = rep.timed(run)
    kms = sum(env.elapsed_ms(4, 5) for env, _ in ctx) / len(ctx)
    for env, io in ctx:
        io.close()
        env.close()
    avg = kms / 1e3 / args.api_steps
    ach = n * ALG_BYTES_API / avg / 1e9
    # the quad API steps (k_env_step_api4; the random opponent's: k_env_step_api4_vs<BLACK>) --
    # GC_NO_QUAD_API=1: the opponent's paired one
    paired = os.environ.get("GC_NO_QUAD_API", "0") not in ("", "0")
    black = env_kw.get("player_color") == "BLACK"
    kern = (("k_env_step_api2_vs" if paired else "k_env_step_api4_vs") + ("<true>" if black else "<false>")
            if env_kw else "k_env_step_api4")
    out = {"value": rep.world_size * n * args.api_steps / dt, "unit": "env_steps/s", "steps": args.api_steps,
           "roofline": {"bound": "hbm", "kernel": kern, "achieved": ach,
                        "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS, "avg_launch_us": avg * 1e6,
                        "alg_bytes_per_board": ALG_BYTES_API, "traffic": None}}
    pa = load_pmc(os.path.join(ROOT, "profiles", "pmc_api_latest.json"))
    kp = (pa or {}).get("kernels", {}).get(kern)
    if kp is None and kern.endswith("<false>"):  # summaries before round 6 dropped the template argument
        kp = (pa or {}).get("kernels", {}).get(kern[:-len("<false>")])
    if kp:  # HBM bytes per launch by PMC (tools/api_pmc.sh), scaled to this run's boards
        out["roofline"]["traffic"] = kp["bytes_per_board"] * n
        out["roofline"]["pmc_source"] = {"file": "profiles/pmc_api_latest.json", "profile": pa.get("profile"),
                                         "bytes_per_board": kp["bytes_per_board"],
                                         "note": "FETCH_SIZE x2 + WRITE_SIZE per launch of the bench's API legs"}
    if env_kw:
        out["env"] = env_kw
    return out


def reference_driver(env, episodes, steps, seed):
    """/root/reference/gym_chess/test/v2/test_benchmark.py:9-43, statement for statement:
    random self-play over env.possible_moves with numpy's global generator."""
    import numpy as np

    np.random.seed(seed)
    total = 0
    t0 = time.perf_counter()
    for _ in range(episodes):
        env.reset()
        for _ in range(steps):
            total += 1
            moves = env.possible_moves
            if not moves:
                break
            move = moves[np.random.choice(np.arange(len(moves)))]
            _, _, done, _ = env.step(env.move_to_action(move))
            if done:
                break
    return total, time.perf_counter() - t0


def single_env_leg(args, rep):
    """configs[0] / the reference's own benchmark (test_benchmark.py: 10 episodes x <= 100
    steps, published 312 us per step for the Rust v2 engine): the chess_v2.py-shaped
    single-board env (gc_env_single_call per step, served by a resident wave through a
    host-mapped mailbox, its result in a host-mapped record: no launch per step).  CPU
    baseline: the same driver and env class over the C oracle's restatement of the same ops
    on one core.  Beside it, one ChessEngine.get_possible_moves call on the start-position
    dict (README.md:372-374 publishes 240 us for the v2 engine), served by the engine's
    resident wave."""
    from gym_chess_amd import codec as C
    from gym_chess_amd.engine import ChessEngine
    from gym_chess_amd.single import ChessEnv

    rp = rep.local[0]
    env = ChessEnv(opponent="none", log=False, device=rp.device)
    reference_driver(env, 1, 10, 1)  # load the kernel
    steps, dt = reference_driver(env, args.single_episodes, 100, 0x5EED)
    out = {"value": dt / steps * 1e6, "unit": "us/step", "higher_is_better": False, "steps": steps,
           "episodes": args.single_episodes, "reference_published_us_per_step": 312.0,
           "form": "one gc_env_single_call per step, served by the resident single-board wave (k_single_server: "
                   "host-mapped mailbox in, device bookkeeping, host-mapped record out; no launch per step)"}
    env.close()
    eng = ChessEngine(rp.device)
    state = dict(board=C.DEFAULT_BOARD, current_player="WHITE", white_king_castle_is_possible=True,
                 white_queen_castle_is_possible=True, black_king_castle_is_possible=True,
                 black_queen_castle_is_possible=True)
    for _ in range(20):
        eng.get_possible_moves(state, "WHITE")
    calls = 500
    t0 = time.perf_counter()
    for _ in range(calls):
        eng.get_possible_moves(state, "WHITE")
    out["engine_get_possible_moves"] = {"value": (time.perf_counter() - t0) / calls * 1e6, "unit": "us/call",
                                        "calls": calls, "reference_published_us_per_call": 240.0,
                                        "state": "DEFAULT_BOARD dict, WHITE",
                                        "form": "one-position call served by the resident engine wave (k_engine_server)"}
    if rep.rank == 0 and rep.world_size == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from oracle_engine import OracleBoard

        cenv = ChessEnv(opponent="none", log=False, backend=OracleBoard())
        cs, cdt = reference_driver(cenv, args.single_episodes, 100, 0x5EED)
        out["cpu_baseline"] = {"value": cdt / cs * 1e6, "unit": "us/step", "cores": 1, "kind": "port",
                               "sample": f"the same driver and env class, {cs} steps over the C oracle's env ops"}
    return out


def variant_legs(args, rep, n):
    """step() throughput of the SURVEY 8f variants at the same batch: the in-kernel random
    opponent (one step = the agent's ply + the opponent's reply) and FIDE rules.  Same timing
    discipline as the main line (one fused launch of --variant-steps steps with the per-step
    trace), plus the launched form (one kernel per step)."""
    from gym_chess_amd.env import BatchedChessEnv

    out = {}
    k = args.variant_steps
    for name, kw in (("opponent_random", dict(opponent="random")), ("rules_fide", dict(rules="fide"))):
        def setup(rp):
            env = BatchedChessEnv(n, device=rp.device, seed=rp.board_seed(args.seed + 7), **kw)
            tb = env.trace_buffer(k)
            env.step_random(max(args.warmup, 200))
            env.rollout_device(k, tb)  # loads the fused kernel
            env.synchronize()
            return env, tb

        ctx = rep.run(setup)
        s0 = [int(e.outputs()["nsteps"].sum()) for e, _ in ctx]

        def run(rp):
            env, tb = ctx[rep.local.index(rp)]
            env.synchronize()
            t0 = time.perf_counter()
            env.rollout_device(k, tb)
            env.synchronize()
            return None, time.perf_counter() - t0

        _, dt = rep.timed(run)
        s1 = [int(e.outputs()["nsteps"].sum()) for e, _ in ctx]
        out[name] = {"value": rep.sum(sum(b - a for a, b in zip(s0, s1))) / dt, "unit": "env_steps/s", "steps": k,
                     "form": "one fused launch (gc_env_rollout_device) with the per-step trace"}
        if args.launched_steps > 0:
            def launched(rp):
                env, _ = ctx[rep.local.index(rp)]
                env.synchronize()
                t0 = time.perf_counter()
                env.step_random(k)
                env.synchronize()
                return None, time.perf_counter() - t0

            s0 = [int(e.outputs()["nsteps"].sum()) for e, _ in ctx]
            _, ldt = rep.timed(launched)
            s1 = [int(e.outputs()["nsteps"].sum()) for e, _ in ctx]
            out[name]["launched_step"] = {"value": rep.sum(sum(b - a for a, b in zip(s0, s1))) / ldt,
                                          "unit": "env_steps/s", "steps": k}
        for e, tb in ctx:
            tb.close()
            e.close()
    return out


def concurrent_leg(args, rep, ctx, n, s_per_step):
    """Replicas measured over a common interval: the headline's K-step
    regions are ~0.1 ms, far below the replicas' barrier skew, so they need not overlap and N
    of them say nothing about contention.  Here every replica repeats the same K-step launch
    R times back to back, R chosen (the same on every rank) so a region lasts >= --concurrent-ms;
    each region's begin / end on CLOCK_MONOTONIC (node-wide) gives the union wall time and the
    fraction of the longest region common to all (min_overlap)."""
    ms = args.concurrent_ms if args.concurrent_ms > 0 else 250.0
    batch = max(1, int(0.01 / (s_per_step * max(args.steps, 1))))  # ~10 ms of launches between clock checks
    s0 = [int(c[0].outputs()["nsteps"].sum()) for c in ctx]
    launches = [0] * len(ctx)

    def run(rp):
        k = rep.local.index(rp)
        env, tb = ctx[k][:2]
        env.synchronize()
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < ms / 1e3:
            for _ in range(batch):
                env.rollout_device(args.steps, tb)
            env.wait_rollout()
            launches[k] += batch
        return None, time.perf_counter() - t0, t0

    _, dt = rep.timed(run)
    ov = rep.last_overlap
    s1 = [int(c[0].outputs()["nsteps"].sum()) for c in ctx]
    steps = rep.sum(sum(b - a for a, b in zip(s0, s1)))
    wall = ov["union_wall_s"] if ov else dt
    return {"value": steps / wall, "unit": "env_steps/s", "launches_per_replica": launches, "steps_per_launch": args.steps,
            "env_steps": steps, "union_wall_s": wall, "max_region_s": dt, "overlap": ov,
            "form": "every replica repeats the headline's K-step launch back to back over a common interval; "
                    "value = all replicas' env.steps / the union of their regions"}


def launched_leg(args, rep, envs, n):
    """The launched form of the same step: one k_env_step2 launch per ply over two
    board-range streams (gc_env_step_random), --launched-steps plies; roofline of k_env_step2
    per ply by HIP events on the env's stream."""
    for e in envs:
        e.step_random(5)  # loads the step kernel
        e.synchronize()
    s0 = [int(e.outputs()["nsteps"].sum()) for e in envs]

    def run(rp):
        env = envs[rep.local.index(rp)]
        env.synchronize()
        t0 = time.perf_counter()
        env.record_event(2)
        env.step_random(args.launched_steps)
        env.record_event(3)
        env.synchronize()
        return None, time.perf_counter() - t0

    _, dt = rep.timed(run)
    s1 = [int(e.outputs()["nsteps"].sum()) for e in envs]
    ply_s = sum(e.elapsed_ms(2, 3) for e in envs) / len(envs) / 1e3 / args.launched_steps
    ach = n * ALG_BYTES_PER_BOARD / ply_s / 1e9
    out = {"value": rep.sum(sum(b - a for a, b in zip(s0, s1))) / dt, "unit": "env_steps/s",
           "steps": args.launched_steps, "ms_per_step": dt * 1e3 / args.launched_steps,
           "roofline": {"bound": "hbm", "kernel": "k_env_step2", "achieved": ach, "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": ach / HBM_PEAK_GBS, "avg_ply_us": ply_s * 1e6,
                        "alg_bytes_per_board": ALG_BYTES_PER_BOARD}}
    pm = load_pmc(PMC_STEP_FILE)
    if pm:
        out["roofline"]["traffic"] = pm.get("bytes_per_launch")
        out["roofline"]["pmc_source"] = {"file": os.path.relpath(PMC_STEP_FILE, ROOT), "profile": pm.get("profile")}
    return out


def main():
    args = parse()
    from gym_chess_amd.env import BatchedChessEnv
    from gym_chess_amd.replicas import Replicas

    devs = os.environ.get("GC_BENCH_DEVICES")  # replica -> device map (tests: several replicas on one GPU)
    rep = Replicas(gpus=args.gpus, devices=[int(d) for d in devs.split(",")] if devs else None).init()
    n = args.boards

    def setup(rp):
        env = BatchedChessEnv(n, device=rp.device, seed=rp.board_seed(args.seed))
        if args.settle > 0:  # into steady state: mid/late-game boards, resets, terminals
            env.rollout(args.settle)
        tb = env.trace_buffer(max(args.steps, 1))
        tbw = env.trace_buffer(max(args.warmup, 1))
        s0, w0 = int(env.outputs()["nsteps"].sum()), env.window_sum()
        # the W untimed warmup steps through the timed region's own call, and nothing after them:
        # the env's counters are read before the warmup, and the timed steps are counted from the
        # trace (a D2H read of the counters between warmup and timed region left the region ~10 us
        # longer: tools/region_probe.py vs bench)
        env.rollout_device(args.warmup, tbw, events=(0, 1))
        env.synchronize()
        return env, tb, tbw, s0, w0

    ctx = rep.run(setup)
    envs = [c[0] for c in ctx]
    rollout_kernel = ROLLOUT_KERNEL[envs[0].rollout_waves()]
    occ = rollout_kernel == "k_env_rollout4" and args.steps >= envs[0].rollout_occ_min_plies()
    if rollout_kernel == "k_env_rollout4":  # <true>: with the window's occupancy filter
        rollout_kernel += "<true>" if occ else "<false>"

    def step(rp):
        env, tb = ctx[rep.local.index(rp)][:2]
        env.synchronize()
        t0 = time.perf_counter()
        env.rollout_device(args.steps, tb, events=(0, 1))  # K env.step() of every board, one launch, per-step trace
        env.wait_rollout()  # the launch's completion word (its last workgroup, host-mapped)
        t1 = time.perf_counter()
        env.synchronize()  # (off the clock: the stream's own completion, reported beside the value)
        return time.perf_counter() - t0, t1 - t0, t0

    synced, dt_max = rep.timed(step)
    dt_synced = rep.max(max(synced))
    region_overlap = rep.last_overlap
    kern_ms = [e.elapsed_ms(0, 1) for e in envs]
    s1 = [int(e.outputs()["nsteps"].sum()) for e in envs]
    w1 = [e.window_sum() for e in envs]
    # env.step() calls in the timed region, from its per-step trace (action -1: the driver's
    # no-move reset, not a step), cross-checked against the env's step counters, which also
    # count the warmup's steps
    steps_local = 0
    for (env, tb, tbw, s0, _), b in zip(ctx, s1):
        tr = tb.fetch(args.steps)
        timed = int((tr["action"] != -1).sum())
        warm = int((tbw.fetch(args.warmup)["action"] != -1).sum()) if args.warmup > 0 else 0
        assert b - s0 == timed + warm, f"step counters {b - s0} != trace {timed} + {warm}"
        assert (tr["done"][-1] <= 1).all() and (tr["reason"][-1] <= 10).all()  # the last ply was written
        steps_local += timed
        del tr
    steps_all = rep.sum(steps_local)
    value = steps_all / dt_max
    mean_window = sum(c[4] + w for c, w in zip(ctx, w1)) / (2.0 * n * len(envs))

    # roofline of the dominant kernel (the fused K-step launch, k_env_rollout4), per launch,
    # from HIP events on the env's stream (the stream it is launched on; mean over this
    # process's replicas): SURVEY §8(d)'s 173 + 8h bytes per board per ply x N x K
    alg = alg_bytes_fused(mean_window)
    launch_s = sum(kern_ms) / len(kern_ms) / 1e3
    achieved = n * args.steps * alg / launch_s / 1e9
    # the PMC passes of the same kernel variant (the filter halves the window's bytes)
    pmc_file = PMC_FILE_LONG if occ and os.path.exists(PMC_FILE_LONG) else PMC_FILE
    pm = load_pmc(pmc_file)
    traffic = pmc_src = valu = None
    if pm:
        # per launch of THIS run: the profiled launch's bytes per board per ply x boards x steps
        bpp = pm.get("bytes_per_board_ply")
        traffic = bpp * n * args.steps if bpp else None
        valu = pm.get("valu")
        pmc_src = {"file": os.path.relpath(pmc_file, ROOT), "profile": pm.get("profile"), "kernel": pm.get("kernel"),
                   "plies_per_launch": pm.get("plies_per_launch"), "bytes_per_board_ply": pm.get("bytes_per_board_ply"),
                   "note": "rocprofv3 PMC passes of the bench command at that launch length (not this process); traffic = "
                           "its FETCH_SIZE x2 + WRITE_SIZE per board per ply (MI355X guide, gfx950 correction) x boards "
                           "x this launch's steps"}

    # what bounds the kernel: "bound" stays the roofline the contract prices it
    # against (HBM), but at frac ~0.4 the launch is not bandwidth-limited -- half its wave cycles
    # wait on the ply's dependency chain (workgroup barriers, LDS and the window's line) while the
    # SIMDs issue well under their peak
    limiter = None
    if valu:
        limiter = {"kind": "dependency-chain latency (4 barriers per ply, role chains Q2 > Q1)",
                   "wait_any_share": valu.get("wait_any_share"), "issue_frac": valu.get("issue_frac"),
                   "hbm_frac": achieved / HBM_PEAK_GBS,
                   "pmc_bytes_vs_alg": (pm.get("bytes_per_board_ply") or 0) / alg if alg else None}

    extra = {}
    if rep.world_size > 1 or args.concurrent_ms > 0:
        extra["concurrent"] = concurrent_leg(args, rep, ctx, n, dt_max / max(args.steps, 1))
    if args.launched_steps > 0:
        extra["launched_step"] = launched_leg(args, rep, envs, n)
    for e, tb, tbw in ((c[0], c[1], c[2]) for c in ctx):
        tb.close()
        tbw.close()
        e.close()
    if args.api_steps > 0:
        extra["api_step"] = api_step_leg(args, rep, n)
        # the random opponent answering inside each step (chess_v2.py:275-288)
        extra["api_step"]["opponent_random"] = api_step_leg(args, rep, n, opponent="random")
        # a BLACK agent: the opponent opens every reset game (chess_v2.py:208-216), windows unbounded
        extra["api_step"]["opponent_random_black"] = api_step_leg(args, rep, n, opponent="random",
                                                                  player_color="BLACK")
    if args.configs1_roots > 0:
        extra["perft_startpos"] = perft_startpos_leg(args, rep)
    if args.single_episodes > 0:
        extra["single_env"] = single_env_leg(args, rep)
    if args.variant_steps > 0:
        extra["variants"] = variant_legs(args, rep, n)
    if args.perft_roots > 0:
        extra["perft"] = perft_leg(args, rep)

    cpu = None
    if rep.rank == 0 and rep.world_size == 1 and not args.no_cpu_baseline:  # N=1 only (contract)
        cpu = cpu_baseline(args)

    if rep.rank == 0:
        line = {
            "metric": "env steps/sec at 65 536 boards per GPU (random-policy self-play to terminal, auto-reset)",
            "value": value,
            "unit": "env_steps/s",
            "n_gpus": rep.world_size,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt_max * 1e3 / args.steps,
            "timed_region_ms": dt_max * 1e3,
            "event_ms_per_step": launch_s * 1e3 / args.steps,
            # the region as rounds 1-3 ended it: at the stream's own completion
            # (hipStreamSynchronize) instead of the completion word
            "stream_sync_end": {"value": steps_all / dt_synced, "ms_per_step": dt_synced * 1e3 / args.steps},
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic (DEFAULT_BOARD starts, Philox uniform policy)",
            "config": {"workload": "configs[2]: 65536 boards/GPU random-policy rollout to terminal, step() throughput",
                       "boards_per_gpu": n, "global_boards": n * rep.world_size,
                       "parallelism": f"replicas{rep.world_size}", "replica_mode": rep.mode,
                       "settle_plies": args.settle,
                       "step_form": f"K steps = one {rollout_kernel} launch (gc_env_rollout_device), "
                                    "per-step trace in HBM", "steps_per_launch": args.steps,
                       "region_end": "the launch's completion word (written to host-mapped memory by its last "
                                     "workgroup after every workgroup's stores: gc_env_wait_rollout); the stream "
                                     "sync follows off the clock"},
            "region_overlap": region_overlap,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": rollout_kernel, "avg_launch_us": launch_s * 1e6,
                         "plies_per_launch": args.steps, "alg_bytes_per_board_ply": alg,
                         "alg_bytes_rule": "SURVEY 8(d) fused rollout ply: 173 + 8h", "mean_window": mean_window,
                         "valu": valu, "pmc_source": pmc_src, "limiter": limiter},
            "cpu_baseline": cpu,
            **extra,
        }
        print(json.dumps(line), flush=True)
    rep.close()


if __name__ == "__main__":
    main()
