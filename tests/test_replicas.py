"""Multi-process (world_size 2, gloo, CPU) coverage of the replica path used by bench.py:
rank seeds, board ranges, barrier, max/sum of per-rank scalars, and that the per-rank
work really is independent (each rank's CPU-oracle rollouts depend only on its own seed)."""
import os
import socket
import sys

import numpy as np
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    sys.path.insert(0, os.path.join(ROOT, "gym-chess_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from gym_chess_amd.replicas import Replicas
    import oracle as O

    r = Replicas().init()
    seed = r.board_seed(0x5EED)
    b0, b1 = r.global_board_range(4)
    st = O.rollout_batch(seed, 0, 4, 60, threads=1)  # this rank's shard, local board ids
    r.barrier()
    out[rank] = dict(seed=seed, range=(b0, b1), steps=int(st[0]), tmax=r.max(float(rank + 1)),
                     ssum=r.sum(float(st[0])))
    r.close()


def test_two_rank_replicas():
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
    res = [out[r] for r in range(world)]
    assert res[0]["seed"] != res[1]["seed"]
    assert res[0]["range"] == (0, 4) and res[1]["range"] == (4, 8)
    assert res[0]["tmax"] == res[1]["tmax"] == 2.0
    assert res[0]["ssum"] == res[1]["ssum"] == res[0]["steps"] + res[1]["steps"]
    # independence: rank 1's shard equals what a lone process with rank 1's seed computes
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    assert int(O.rollout_batch(res[1]["seed"], 0, 4, 60, threads=1)[0]) == res[1]["steps"]


def test_single_process_defaults():
    sys.path.insert(0, os.path.join(ROOT, "gym-chess_amd"))
    from gym_chess_amd.replicas import Replicas

    r = Replicas(world_size=1, rank=0, local_rank=0).init()
    assert r.board_seed(7) == 7 and r.max(3.5) == 3.5 and r.sum(2.0) == 2.0
    r.barrier()
    r.close()
    assert np.uint64(Replicas(world_size=8, rank=7).board_seed(1)) == np.uint64(1 + (7 << 40))
