#!/usr/bin/env python3
"""Benchmark: env.step() throughput of the batched chess env on MI355X.

Workload (BASELINE.json configs[2], the metric's config): 65 536 boards per GPU, random-
policy self-play to terminal with auto-reset -- the test_benchmark.py driver
(/root/reference/gym_chess/test/v2/test_benchmark.py:9-43) vectorised.  One "step" = one
env.step() on every board: one launch of the one-ply step kernel (k_env_step<true>:
apply the policy's action with the full chess_v2.py step bookkeeping, generate the next
legal set, mate/3-fold/move-cap, pick the next action, reset finished boards).  State,
repetition windows and outputs stay in HBM; nothing crosses PCIe in the timed region.

  python bench.py [--gpus N --steps K --warmup W --boards B]
  multi-GPU: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
  (one process per GPU, boards sharded, no data-path collective: "scaling": "weak")

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

# algorithmic bytes per board per step of k_env_step<true> (DESIGN.md "Roofline"):
#   state 7x8 B bitboards + 4 B meta, read + write            120
#   action read + next-action write (u16)                         4
#   Philox draw counter read + write                               8
#   nsteps counter read + write                                    8
#   outputs reward i32 + done u8 + reason u8                        6
#   repetition window append (4 B key + 56 B board)              60 (reversible plies only)
#   repetition window scan: 4 B per stored key                  4*h
FIXED_BYTES = 120 + 4 + 8 + 8 + 6


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=400)
    ap.add_argument("--boards", type=int, default=65536)
    ap.add_argument("--seed", type=int, default=0x5EED + 3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-boards", type=int, default=32768)
    ap.add_argument("--cpu-sample-plies", type=int, default=300)
    ap.add_argument("--fused-plies", type=int, default=100, help="also time the fused rollout kernel (0 = skip)")
    return ap.parse_args()


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    pg = None
    if world > 1:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)  # barrier + timing max only
        pg = dist
    return world, rank, local, pg


def barrier(pg):
    if pg is not None:
        pg.barrier()


def allmax(pg, x):
    if pg is None:
        return x
    import torch

    t = torch.tensor([float(x)], dtype=torch.float64)
    pg.all_reduce(t, op=pg.ReduceOp.MAX)
    return float(t.item())


def allsum(pg, x):
    if pg is None:
        return x
    import torch

    t = torch.tensor([float(x)], dtype=torch.float64)
    pg.all_reduce(t, op=pg.ReduceOp.SUM)
    return float(t.item())


def cpu_baseline(args):
    """Oracle (C restatement of lib.rs + chess_v2.py, test infrastructure) on host cores:
    the same random self-play driver on a bounded sample of boards."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    threads = max(1, min(16, os.cpu_count() or 1))
    O.lib()
    t0 = time.perf_counter()
    st = O.rollout_batch(args.seed, 0, args.cpu_sample_boards, args.cpu_sample_plies, threads=threads)
    dt = time.perf_counter() - t0
    steps = int(st[0])
    return {
        "value": steps / dt,
        "unit": "env_steps/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{args.cpu_sample_boards} boards x {args.cpu_sample_plies} plies random self-play "
        f"({steps} env.step calls, {dt:.1f} s) with the C oracle restating lib.rs + chess_v2.py",
    }


def main():
    args = parse()
    world, rank, local, pg = dist_setup(args)
    from gym_chess_amd.env import BatchedChessEnv

    n = args.boards
    env = BatchedChessEnv(n, device=local, seed=args.seed + (rank << 40))
    # warmup: also moves the batch off the all-startpos state toward steady-state play
    env.step_random(args.warmup)
    env.synchronize()
    s0 = int(env.outputs()["nsteps"].sum())
    w0 = env.window_sum()
    barrier(pg)
    env.synchronize()
    t0 = time.perf_counter()
    env.record_event(0)
    env.step_random(args.steps)
    env.record_event(1)
    env.synchronize()
    t1 = time.perf_counter()
    barrier(pg)
    dt = t1 - t0
    dt_max = allmax(pg, dt)
    kern_ms = env.elapsed_ms(0, 1)
    s1 = int(env.outputs()["nsteps"].sum())
    w1 = env.window_sum()
    steps_local = s1 - s0
    steps_all = allsum(pg, steps_local)
    value = steps_all / dt_max

    # roofline of the dominant kernel (k_env_step<true>), per launch
    mean_h = 0.5 * (w0 + w1) / n
    bytes_per_launch = n * (FIXED_BYTES + 60 + 4 * mean_h)  # append bound: every ply reversible
    avg_launch_s = kern_ms / 1e3 / args.steps
    achieved = bytes_per_launch / avg_launch_s / 1e9
    traffic = None
    tf = os.path.join(ROOT, "profiles", "pmc_traffic_latest.json")
    if os.path.exists(tf):
        try:
            traffic = json.load(open(tf)).get("bytes_per_launch")
        except Exception:
            traffic = None

    extra = {}
    if args.fused_plies > 0:
        env.synchronize()
        f0 = time.perf_counter()
        env.record_event(2)
        st, _ = env.rollout(args.fused_plies)
        env.record_event(3)
        env.synchronize()
        f1 = time.perf_counter()
        fsteps = allsum(pg, float(st[0]))
        fdt = allmax(pg, f1 - f0)
        extra["fused_rollout"] = {"value": fsteps / fdt, "unit": "env_steps/s", "plies_per_launch": args.fused_plies,
                                  "kernel_ms": env.elapsed_ms(2, 3)}

    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args)

    if rank == 0:
        line = {
            "metric": "env steps/sec at 65 536 boards per GPU (random-policy self-play to terminal, auto-reset)",
            "value": value,
            "unit": "env_steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt_max * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic (DEFAULT_BOARD starts, Philox uniform policy)",
            "config": {"workload": "configs[2]: 65536 boards/GPU random-policy rollout to terminal, step() throughput",
                       "boards_per_gpu": n, "global_boards": n * world, "parallelism": f"replicas{world}"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": "k_env_step<true>", "avg_launch_us": avg_launch_s * 1e6,
                         "alg_bytes_per_board": FIXED_BYTES + 60 + 4 * mean_h, "mean_window": mean_h},
            "cpu_baseline": cpu,
            **extra,
        }
        print(json.dumps(line), flush=True)
    if pg is not None:
        pg.destroy_process_group()


if __name__ == "__main__":
    main()
