"""GPU: several replicas in one process (bench.py --gpus N without a launcher; SURVEY §8e
"one host thread + one handle per device").  On a 1-GPU lease the replicas share device 0:
what is checked is that concurrent handles driven from concurrent host threads leave every
board's trajectory exactly as a lone handle with the same seed plays it."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_two_handles_two_threads_equal_lone_runs():
    from gym_chess_amd.env import BatchedChessEnv
    from gym_chess_amd.replicas import Replicas

    n, plies, seed = 4096, 300, 0x5EED + 3
    rep = Replicas(gpus=2, devices=[0, 0]).init()
    envs = rep.run(lambda rp: BatchedChessEnv(n, device=rp.device, seed=rp.board_seed(seed)))

    def go(rp):
        e = envs[rp.index]
        e.rollout(100)
        e.step_random(plies)
        e.synchronize()
        return e.boards(), e.outputs(), 0.0

    res = rep.run(lambda rp: go(rp))
    for rp, (bm, out, _) in zip(rep.local, res):
        lone = BatchedChessEnv(n, device=0, seed=rp.board_seed(seed))
        lone.rollout(100)
        lone.step_random(plies)
        b, m = lone.boards()
        o = lone.outputs()
        assert (bm[0] == b).all() and (bm[1] == m).all(), rp.index
        for k in ("reward", "done", "reason", "next_action", "nsteps"):
            assert (out[k] == o[k]).all(), (rp.index, k)
        lone.close()
    # the two replicas play different games (distinct Philox keys)
    assert (res[0][0][0] != res[1][0][0]).any()
    for e in envs:
        e.close()


def test_multi_device_env_on_one_gpu():
    from gym_chess_amd.env import BatchedChessEnv, MultiDeviceChessEnv

    n, seed = 1024, 99
    import os

    # inside a launched job (WORLD_SIZE / RANK set) the device_ids contract still holds
    saved = {k: os.environ.get(k) for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    os.environ.update(WORLD_SIZE="2", RANK="1", LOCAL_RANK="1")
    try:
        me = MultiDeviceChessEnv(n, device_ids=(0, 0), seed=seed)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    assert me.total_boards == 2 * n and me.rep.mode == "threads"
    st = me.rollout(200)
    me.set_streams(2)  # forwarded to every env
    me.step_random(50)
    b, m = me.boards()
    ref = np.zeros(8, dtype=np.uint64)
    for r in range(2):
        lone = BatchedChessEnv(n, device=0, seed=me.rep.local[r].board_seed(seed))
        s, _ = lone.rollout(200)
        ref += s
        lone.step_random(50)
        lb, lm = lone.boards()
        assert (b[r * n:(r + 1) * n] == lb).all() and (m[r * n:(r + 1) * n] == lm).all()
        lone.close()
    assert (st == ref).all()
    me.close()


def test_bench_threaded_two_replicas_line():
    """bench.py --gpus 2 in one process on the one GPU (GC_BENCH_DEVICES=0,0): the JSON line
    reports n_gpus 2, global_boards 2 x boards, replica_mode threads."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, GC_BENCH_DEVICES="0,0")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "20", "--warmup",
                          "5", "--settle", "300", "--boards", "8192", "--perft-roots", "0", "--variant-steps", "0",
                          "--no-cpu-baseline", "--launched-steps", "0"], capture_output=True, text=True, env=env,
                         timeout=300, check=True)
    line = json.loads(out.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["config"]["global_boards"] == 2 * 8192
    assert line["config"]["replica_mode"] == "threads" and line["value"] > 0
    # the replicas' common-interval leg ran concurrently
    ov = line["concurrent"]["overlap"]
    assert ov["replicas"] == 2 and ov["min_overlap"] >= 0.9 and line["concurrent"]["max_region_s"] >= 0.2, ov


def test_bench_torchrun_two_ranks_line():
    """The driver's multi-GPU launch shape, rehearsed on the one GPU: python -m
    torch.distributed.run --nproc-per-node 2 bench.py --gpus 2 (GC_BENCH_DEVICES=0,0 puts both
    ranks on device 0): one process per rank, the file-group barrier and max / sum, and ONE
    JSON line from rank 0 with n_gpus 2, global_boards 2 x boards, replica_mode processes."""
    import json
    import os
    import socket
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    env = dict(os.environ, GC_BENCH_DEVICES="0,0")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(root, "bench.py"),
                          "--gpus", "2", "--steps", "20", "--warmup", "5", "--settle", "300", "--boards", "8192",
                          "--perft-roots", "0", "--variant-steps", "0", "--api-steps", "0", "--single-episodes", "0",
                          "--no-cpu-baseline", "--launched-steps", "0"], capture_output=True, text=True, env=env,
                         timeout=240, check=True)
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["config"]["global_boards"] == 2 * 8192
    assert line["config"]["replica_mode"] == "processes" and line["value"] > 0
    # the two ranks' >= 200 ms regions overlap >= 90 % on the node's clock
    ov = line["concurrent"]["overlap"]
    assert ov["replicas"] == 2 and ov["min_overlap"] >= 0.9 and line["concurrent"]["max_region_s"] >= 0.2, ov
    assert line["region_overlap"]["replicas"] == 2
