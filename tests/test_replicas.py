"""Multi-replica coverage on the CPU (no GPU): the replica path bench.py uses.

* processes (world_size 2, one process per rank as torch.distributed.run starts them): rank
  seeds, board ranges, barrier, max / sum of per-rank scalars through the file group (the
  default, no torch) and through gloo (GC_REPLICA_BACKEND=gloo); per-rank work is
  independent (each rank's CPU-oracle rollouts depend only on its own seed).
* threads (`bench.py --gpus N` without a launcher): N replicas in one process, one thread
  each, results in replica order, exceptions propagated, the timed region's max.
"""
import multiprocessing as mp
import os
import socket
import sys
import time

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, backend, out):
    sys.path.insert(0, os.path.join(ROOT, "gym-chess_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), GC_REPLICA_BACKEND=backend, GC_REPLICA_KEY=f"test_{port}")
    from gym_chess_amd.replicas import Replicas
    import oracle as O

    r = Replicas(gpus=world).init()
    (rp,) = r.local
    seed = rp.board_seed(0x5EED)
    b0, b1 = rp.board_range(4)
    st = O.rollout_batch(seed, 0, 4, 60, threads=1)  # this rank's shard, local board ids
    r.barrier()
    res = dict(seed=seed, range=(b0, b1), steps=int(st[0]), tmax=r.max(float(rank + 1)), ssum=r.sum(float(st[0])),
               device=rp.device, mode=r.mode)
    # many rounds back to back: a fast rank may run one round ahead of a slow one
    acc = [r.sum(float(k * (rank + 1))) for k in range(50)]
    res["acc_ok"] = acc == [float(3 * k) for k in range(50)]
    # ranks whose timed fn returns different shapes (rank 0 a begin time, rank 1 none) still issue
    # the same collectives: no deadlock, no overlap claimed, the max still taken
    _, dt = r.timed(lambda rp: (None, 0.5 + rank, time.perf_counter()) if rank == 0 else (None, 0.5 + rank))
    res["mixed_ok"] = dt == 1.5 and r.last_overlap is None
    _, dt = r.timed(lambda rp: (None, 0.25, time.perf_counter()))
    res["spans_ok"] = r.last_overlap is not None and r.last_overlap["replicas"] == 2
    r.close()
    out.put((rank, res))


@pytest.mark.parametrize("backend", ["file", "gloo"])
def test_two_rank_replicas(backend):
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, backend, q)) for r in range(world)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=300) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    res = [got[r] for r in range(world)]
    assert res[0]["mode"] == "processes" and [x["device"] for x in res] == [0, 1]
    assert res[0]["seed"] != res[1]["seed"]
    assert res[0]["range"] == (0, 4) and res[1]["range"] == (4, 8)
    assert res[0]["tmax"] == res[1]["tmax"] == 2.0
    assert res[0]["ssum"] == res[1]["ssum"] == res[0]["steps"] + res[1]["steps"]
    assert res[0]["acc_ok"] and res[1]["acc_ok"]
    assert all(x["mixed_ok"] and x["spans_ok"] for x in res)
    # independence: rank 1's shard equals what a lone process with rank 1's seed computes
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    assert int(O.rollout_batch(res[1]["seed"], 0, 4, 60, threads=1)[0]) == res[1]["steps"]


def test_gpus_mismatch_with_launcher(monkeypatch):
    sys.path.insert(0, os.path.join(ROOT, "gym-chess_amd"))
    from gym_chess_amd.replicas import Replicas

    monkeypatch.setenv("WORLD_SIZE", "2")
    with pytest.raises(ValueError):
        Replicas(gpus=8)


def test_threaded_replicas(monkeypatch):
    """--gpus 3 in one process: one thread per replica on devices 0..2, the oracle standing in
    for each replica's device work; results in replica order == the same work done serially."""
    sys.path.insert(0, os.path.join(ROOT, "gym-chess_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    from gym_chess_amd.replicas import Replicas
    import oracle as O

    r = Replicas(gpus=3).init()
    assert r.mode == "threads" and r.world_size == 3 and [x.device for x in r.local] == [0, 1, 2]

    def work(rp):
        t0 = time.perf_counter()
        st = O.rollout_batch(rp.board_seed(0x5EED), 0, 4, 60, threads=1)
        return (rp.index, int(st[0])), time.perf_counter() - t0

    res, dt = r.timed(work)
    assert [x[0] for x in res] == [0, 1, 2] and dt > 0
    serial = [int(O.rollout_batch(rp.board_seed(0x5EED), 0, 4, 60, threads=1)[0]) for rp in r.local]
    assert [x[1] for x in res] == serial
    assert r.sum(5.0) == 5.0 and r.max(2.0) == 2.0  # one process: nothing to reduce across

    def boom(rp):
        if rp.index == 1:
            raise RuntimeError("replica 1 failed")
        return rp.index

    with pytest.raises(RuntimeError, match="replica 1"):
        r.run(boom)
    r.close()


def test_single_process_defaults(monkeypatch):
    sys.path.insert(0, os.path.join(ROOT, "gym-chess_amd"))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    from gym_chess_amd.replicas import Replica, Replicas

    r = Replicas().init()
    assert r.world_size == 1 and r.local[0].board_seed(7) == 7 and r.max(3.5) == 3.5 and r.sum(2.0) == 2.0
    r.barrier()
    r.close()
    assert np.uint64(Replica(7, 0).board_seed(1)) == np.uint64(1 + (7 << 40))


def test_forced_thread_mode_under_a_launcher(monkeypatch):
    """MultiDeviceChessEnv's replicas stay threads inside a launched job."""
    sys.path.insert(0, os.path.join(ROOT, "gym-chess_amd"))
    from gym_chess_amd.replicas import Replicas

    monkeypatch.setenv("WORLD_SIZE", "4")
    monkeypatch.setenv("RANK", "3")
    r = Replicas(gpus=2, devices=(0, 0), mode="threads").init()
    assert r.mode == "threads" and r.world_size == 2 and [x.index for x in r.local] == [0, 1]
    assert r.run(lambda rp: r.local.index(rp)) == [0, 1]
    r.close()
    with pytest.raises(ValueError):
        Replicas(mode="mpi")


def test_file_group_key_changes_with_restart(monkeypatch, tmp_path):
    """a torchrun worker restart (same launcher pid and port) must not read the
    previous attempt's rank records: the restart count is part of the group key."""
    sys.path.insert(0, os.path.join(ROOT, "gym-chess_amd"))
    import gym_chess_amd.replicas as R

    monkeypatch.setattr(R.tempfile, "gettempdir", lambda: str(tmp_path))
    monkeypatch.delenv("GC_REPLICA_KEY", raising=False)
    monkeypatch.setenv("MASTER_PORT", "29555")
    dirs = []
    for restart in ("0", "1"):
        monkeypatch.setenv("TORCHELASTIC_RESTART_COUNT", restart)
        r = R.Replicas(world_size=2, rank=0, local_rank=0)
        r.init()
        dirs.append(r._group.dir)
    assert dirs[0] != dirs[1]


def _overlap_worker(rank, world, port, out):
    sys.path.insert(0, os.path.join(ROOT, "gym-chess_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), GC_REPLICA_KEY=f"ovl_{port}")
    from gym_chess_amd.replicas import Replicas

    r = Replicas(gpus=world).init()

    def region(rp):  # a 300 ms region, the second rank starting 30 ms late
        time.sleep(0.03 * rank)
        t0 = time.perf_counter()
        time.sleep(0.3)
        return rank, time.perf_counter() - t0, t0

    res, dt = r.timed(region)
    out.put((rank, dict(res=res, dt=dt, ov=r.last_overlap)))
    r.close()


def test_two_rank_region_overlap():
    """the ranks' timed regions are gathered on CLOCK_MONOTONIC and their
    overlap reported -- two 300 ms regions 30 ms apart overlap ~90 %, seen alike by both ranks."""
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_overlap_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank in range(world):
        ov = got[rank]["ov"]
        assert ov["replicas"] == 2
        assert 0.8 < ov["min_overlap"] < 0.95, ov
        assert 0.02 < ov["begin_skew_s"] < 0.1, ov
        assert 0.32 < ov["union_wall_s"] < 0.5, ov
    assert got[0]["ov"] == got[1]["ov"]


def test_overlap_math():
    from gym_chess_amd.replicas import overlap

    o = overlap([(0.0, 1.0), (0.5, 1.5)])
    assert o["union_wall_s"] == 1.5 and o["min_overlap"] == 0.5 and o["begin_skew_s"] == 0.5
    assert overlap([(0.0, 1.0), (2.0, 3.0)])["min_overlap"] == 0.0
    assert overlap([(1.0, 2.0)] * 3)["min_overlap"] == 1.0
