"""GPU: step() on device buffers (gc_env_step_device) -- the reference's call shape
(chess_v2.py:219-294: external action in; reward, done, info, observation out; the rebuilt
possible_actions, 333-335) for a policy on the GPU."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _mask_bits(raw):
    n = raw.shape[0]
    bits = np.unpackbits(raw[:, :64].view(np.uint8).reshape(n, 64, 8), axis=2, bitorder="little")
    out = np.zeros((n, 4101), dtype=bool)
    out[:, :4096] = bits.reshape(n, 4096).astype(bool)
    for c in range(4):
        out[:, 4096 + c] = (raw[:, 64] >> np.uint64(c)) & np.uint64(1) != 0
    return out


@pytest.mark.parametrize("opponent", ["none", "random"])
def test_step_device_equals_host_step(oracle, opponent):
    """Same external actions (legal and invalid) into two envs: device-buffer step == host
    step, ply by ply: outputs, states, and the mask / obs / count describe the new states."""
    from gym_chess_amd.env import BatchedChessEnv

    n = 300
    a = BatchedChessEnv(n, device=0, seed=17, opponent=opponent)
    b = BatchedChessEnv(n, device=0, seed=17, opponent=opponent)
    io = a.device_io(pick=False)
    act_buf = a.device_io(mask=False, obs=False, count=False, pick=True, select=False)  # action upload slot
    rng = np.random.RandomState(3)
    for ply in range(120):
        lists = b.possible_actions()
        acts = np.array([l[rng.randint(len(l))] if l and rng.rand() > 0.05 else rng.randint(4101) for l in lists],
                        dtype=np.uint16)
        act_buf.upload_actions(acts)
        a.step_device(io, actions=act_buf.ptr["pick"])
        rw, dn, why = b.step(acts)
        o = io.fetch()
        assert (o["reward"] == rw).all() and (o["done"].astype(bool) == dn).all() and (o["reason"] == why).all(), ply
        bb, bm = b.boards()
        ab, am = a.boards()
        assert (ab == bb).all() and (am == bm).all(), ply
        assert (o["obs"] == bb).all(), ply
        assert (_mask_bits(o["mask"]) == b.legal_mask()).all(), ply
        assert (o["count"] == np.array([len(x) for x in b.possible_actions()])).all(), ply
        if dn.any():
            a.reset(dn.astype(np.uint8))
            b.reset(dn.astype(np.uint8))


def test_step_device_autoreset_pick_loop_vs_oracle(oracle):
    """actions = the previous call's pick, auto-reset on: the random self-play driver with the
    pick in the mask's (action-id) order, ply by ply == the oracle's, on every board until it
    first meets a position with no legal move (there the driver resets without a step, while
    step() reports an invalid action)."""
    from gym_chess_amd.env import BatchedChessEnv

    n, plies, seed = 256, 400, 2718
    env = BatchedChessEnv(n, device=0, seed=seed)
    io = env.device_io()
    refs = [oracle.rollout_trace(seed, i, plies + 1, order="action") for i in range(n)]
    # the env's own first picks are the self-play policy's (move-set order): start the loop
    # from the action-id-order ones
    io.upload_actions(np.array([r["action"][0] for r in refs], dtype=np.uint16))
    live = np.ones(n, dtype=bool)
    checked = 0
    for p in range(plies):
        env.step_device(io, autoreset=True)
        o = io.fetch("reward", "done", "reason", "pick")
        live &= np.array([r["reason"][p] != 4 and r["action"][p] >= 0 for r in refs])
        rr = np.array([r["reward"][p] for r in refs])
        rd = np.array([r["done"][p] for r in refs])
        nx = np.array([r["action"][p + 1] for r in refs])
        assert (o["reward"][live] == rr[live]).all() and (o["done"][live] == rd[live]).all(), p
        ok = live & (nx >= 0)
        assert (o["pick"][ok] == nx[ok]).all(), p
        checked += int(live.sum())
    assert checked > n * plies // 2


def test_obs_of_weird_boards(oracle):
    """The byte-plane observation writer on boards with every piece id in every square class."""
    from conftest import random_positions
    from gym_chess_amd.env import BatchedChessEnv

    boards, metas = random_positions(128, 99)
    env = BatchedChessEnv(128, device=0, seed=1)
    env.set_states(boards, metas)
    io = env.device_io(mask=False, count=False, pick=False)
    act = env.device_io(mask=False, obs=False, count=False, pick=True, select=False)
    act.upload_actions(np.full(128, 4100, dtype=np.uint16))  # RESIGN: invalid, state unchanged
    env.step_device(io, actions=act.ptr["pick"])
    o = io.fetch()
    assert (o["reason"] == 6).all() and (o["obs"] == boards).all()


@pytest.mark.parametrize("opponent,autoreset", [("none", False), ("none", True), ("random", False)])
def test_step_device_weird_boards_equal_host_step(oracle, autoreset, opponent):
    """Fuzz positions (several / no kings, pawns on back ranks, > 16 pieces, rights without
    rooks): the device-buffer step (the quad kernels: quick_legal validation, regen of kept
    states, the per-piece fallback of a both-checked or > 16-piece board; with the random
    opponent its reply too) == the host step ply by ply, with the mask / obs / count of every
    board; with auto-reset, the reset boards' too (the host reset takes a policy draw that the
    device's does not, so the random opponent's auto-reset form is checked against the paired
    kernel below and against the oracle in test_step_device_random_opponent_vs_oracle)."""
    from conftest import random_positions
    from gym_chess_amd.env import BatchedChessEnv

    n = 1000
    boards, metas = random_positions(n, 4242)
    a = BatchedChessEnv(n, device=0, seed=5, opponent=opponent)
    b = BatchedChessEnv(n, device=0, seed=5, opponent=opponent)
    assert a.paired()
    a.set_states(boards, metas)
    b.set_states(boards, metas)
    io = a.device_io(pick=False)
    act_buf = a.device_io(mask=False, obs=False, count=False, pick=True, select=False)
    rng = np.random.RandomState(8)
    reasons = set()
    for ply in range(6):
        lists = b.possible_actions()
        acts = np.array([l[rng.randint(len(l))] if l and rng.rand() > 0.2 else rng.randint(4101) for l in lists],
                        dtype=np.uint16)
        act_buf.upload_actions(acts)
        a.step_device(io, actions=act_buf.ptr["pick"], autoreset=autoreset)
        rw, dn, why = b.step(acts)
        if autoreset and dn.any():
            b.reset(dn.astype(np.uint8))
        reasons |= set(int(x) for x in why)
        o = io.fetch()
        assert (o["reward"] == rw).all() and (o["done"].astype(bool) == dn).all() and (o["reason"] == why).all(), ply
        bb, bm = b.boards()
        ab, am = a.boards()
        assert (ab == bb).all() and (am == bm).all(), ply
        assert (o["obs"] == bb).all(), ply
        assert (_mask_bits(o["mask"]) == b.legal_mask()).all(), ply
        assert (o["count"] == np.array([len(x) for x in b.possible_actions()])).all(), ply
    assert {0, 6}.issubset(reasons), reasons


@pytest.mark.parametrize("color", ["WHITE", "BLACK"])
@pytest.mark.parametrize("autoreset", [False, True])
def test_step_device_random_opponent_vs_oracle(oracle, color, autoreset):
    """The random opponent's device-buffer step -- the quad kernel k_env_step_api4_vs for both
    agent colours (gc_env_step_device2's dispatch; a BLACK agent's reset opening taken from the
    openings cache, k_init_open_cache): the agent's half-ply, the reply -- in lockstep with the
    oracle env (chess_v2.py:219-294 with the opponent policy): rewards / done / reasons,
    states, observation, mask, count; and every pick == the k-th legal action in action-id
    order for the oracle's draw counter.  Actions: mostly the previous pick, some other legal
    ones, some invalid; 200 boards (a partial last workgroup)."""
    from gym_chess_amd.env import BatchedChessEnv

    n, plies, seed = 200, 150, 0x0A11
    env = BatchedChessEnv(n, device=0, seed=seed, opponent="random", player_color=color)
    assert env.paired()
    io = env.device_io()  # pick = the env's creation-time picks (one draw each)
    ors = [oracle.OracleEnv(opponent=1, agent_white=color == "WHITE", seed=seed, board=i) for i in range(n)]
    for o in ors:
        o.pick()
    act_buf = env.device_io(mask=False, obs=False, count=False, pick=True, select=False)
    rng = np.random.RandomState(12)
    prev = io.fetch("pick")["pick"].astype(np.int64)
    for ply in range(plies):
        acts = prev.copy()
        for i, o in enumerate(ors):
            r = rng.rand()
            if r < 0.1:
                acts[i] = rng.randint(4101)
            elif r < 0.3 and o.moves():
                mv = o.moves()
                acts[i] = mv[rng.randint(len(mv))]
            elif acts[i] == 0xFFFF:
                acts[i] = 0
        act_buf.upload_actions(acts.astype(np.uint16))
        env.step_device(io, actions=act_buf.ptr["pick"], autoreset=autoreset)
        out = io.fetch()
        b, m = env.boards()
        ends = np.zeros(n, dtype=np.uint8)
        for i, o in enumerate(ors):
            rc, rw, dn, why = o.step(int(acts[i]))
            if rc == 1:  # both kings checked (kings are capturable, Q7): the engine raises, the env ends
                dn, why = 1, 5
            assert (rw, dn, why) == (int(out["reward"][i]), int(out["done"][i]), int(out["reason"][i])), (ply, i)
            if dn and autoreset:
                o.reset()
            ob, om = o.state()
            assert (b[i] == ob).all() and list(m[i]) == list(om), (ply, i)
            assert (out["obs"][i] == ob).all(), (ply, i)
            legal = sorted(o.moves())
            got = np.nonzero(_mask_bits(out["mask"][i:i + 1])[0])[0].tolist()
            assert got == legal and out["count"][i] == len(legal), (ply, i)
            if legal:
                k = oracle.policy_index(seed, i, o.draw, len(legal))
                assert out["pick"][i] == legal[k], (ply, i)
                o.pick()  # the pick's draw
            else:
                assert out["pick"][i] == 0xFFFF
            if dn and not autoreset:
                ends[i] = 1
        if ends.any():  # the host reset picks a policy action too (one more draw)
            env.reset(ends)
            for i in np.nonzero(ends)[0]:
                ors[i].reset()
                ors[i].pick()
        prev = env.outputs()["next_action"].astype(np.int64) if ends.any() else out["pick"].astype(np.int64)


@pytest.mark.parametrize("kind", ["quad", "opponent", "fide"])
def test_step_device_mask_stride(kind):
    """A padded mask row stride (gc_env_step_device2's argument) moves only the rows: envs stepped
    alike, one with packed rows and one with N + 37 and N + 512 words between rows, give equal
    masks and outputs -- on the quad API step, the random opponent's paired step and the FIDE
    one-lane step."""
    from gym_chess_amd.env import BatchedChessEnv

    n = 1024
    kw = {"quad": {}, "opponent": {"opponent": "random"}, "fide": {"rules": "fide"}}[kind]
    envs = [BatchedChessEnv(n, device=0, seed=31, **kw) for _ in range(3)]
    ios = [e.device_io(mask_stride=st) for e, st in zip(envs, (n, n + 37, n + 512))]
    assert [io.mask_stride for io in ios] == [n, n + 37, n + 512]
    for ply in range(40):
        outs = []
        for e, io in zip(envs, ios):
            e.step_device(io, autoreset=True)
            outs.append(io.fetch())
        for o in outs[1:]:
            for k in outs[0]:
                assert (o[k] == outs[0][k]).all(), (ply, k)
        assert outs[0]["mask"].shape == (n, 65)


@pytest.mark.parametrize("color", ["WHITE", "BLACK"])
@pytest.mark.parametrize("start", ["weird", "settled"])
def test_quad_opponent_api_equals_paired(start, color):
    """The random opponent's quad API step (k_env_step_api4_vs) == the paired one
    (k_env_step_api2_vs, GC_NO_QUAD_API=1) ply by ply with auto-reset: outputs, picks, mask, obs,
    count and states -- on fuzz positions (> 16 pieces, both kings checked, no kings) and on
    boards settled by 300 plies of play; a BLACK agent's resets open with the opponent's move
    (the quads take the opening's position and moves from k_init_open_cache)."""
    import os

    from conftest import random_positions
    from gym_chess_amd.env import BatchedChessEnv

    n = 1000 if start == "weird" else 4096
    envs = [BatchedChessEnv(n, device=0, seed=77, opponent="random", player_color=color) for _ in range(2)]
    if start == "weird":
        boards, metas = random_positions(n, 5151)
        for e in envs:
            e.set_states(boards, metas)
    else:
        for e in envs:
            e.rollout(300)
    ios = [e.device_io() for e in envs]
    acts = envs[0].device_io(mask=False, obs=False, count=False, pick=True, select=False)
    rng = np.random.RandomState(4)
    reasons = set()
    for ply in range(40):
        lists = envs[0].possible_actions()
        a = np.array([l[rng.randint(len(l))] if l and rng.rand() > 0.1 else rng.randint(4101) for l in lists],
                     dtype=np.uint16)
        acts.upload_actions(a)
        outs = []
        for k, (e, io) in enumerate(zip(envs, ios)):
            if k:
                os.environ["GC_NO_QUAD_API"] = "1"
            try:
                e.step_device(io, actions=acts.ptr["pick"], autoreset=True)
                outs.append(io.fetch())
            finally:
                os.environ.pop("GC_NO_QUAD_API", None)
        for key in outs[0]:
            assert (outs[0][key] == outs[1][key]).all(), (ply, key, np.nonzero(outs[0][key] != outs[1][key])[0][:4])
        b0, m0 = envs[0].boards()
        b1, m1 = envs[1].boards()
        assert (b0 == b1).all() and (m0 == m1).all(), ply
        reasons |= set(int(x) for x in outs[0]["reason"])
    assert {0, 6}.issubset(reasons), reasons
