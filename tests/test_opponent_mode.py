"""Opponent mode (chess_v2.py:167-181 opponent policy, 208-216 BLACK opening, 275-292 reply,
LOSS/WIN terms, move_count cadence) against the reference ChessEnvV2's own traces.

tests/golden/v2_opp_traces.json.gz: the reference env (make_golden.trace_opp) with a callable
opponent playing the device policy (Philox rank over the legal list, k-th in action-id
order); the agent draws from the same counter.  The oracle (CPU), the host build of the
device code (CPU) and the HIP env (GPU) must reproduce every step.
"""
import numpy as np
import pytest

from conftest import load_golden


def _init(t):
    from gym_chess_amd import codec as C
    import oracle as O

    return O.DEFAULT_BOARD if t["initial_board"] is None else C.text_to_board(t["initial_board"])


def test_oracle_opponent_mode_vs_reference_traces(oracle):
    from gym_chess_amd import codec as C

    n = 0
    for t in load_golden("v2_opp_traces.json.gz"):
        env = oracle.OracleEnv(_init(t), opponent=1, agent_white=t["color"] == "WHITE", seed=t["seed"],
                               board=t["board"])
        for s in t["steps"]:
            if s["kind"] == "reset":
                env.reset()
                assert env.draw == s["draw"]
                continue
            a = env.pick()
            assert a == s["action"]
            rc, rw, dn, why = env.step(a)
            if s["kind"] == "error":
                assert rc == 1
                continue
            if s["kind"] == "opp_no_move":
                assert why == 9
                continue
            assert rc == 0 and rw == s["reward"] and bool(dn) == s["done"], s
            b, m = env.state()
            assert C.board_to_text(b) == s["board"] and list(m[:7]) == s["meta"] and m[7] == s["move_count"], s
            assert len(env.moves()) == s["n_moves"] and env.draw == s["draw"]
            n += 1
    assert n > 3000


def test_oracle_opponent_rollout_matches_env_driver(oracle):
    """rollout_trace(opponent=1) == stepping OracleEnv with the same driver."""
    for white in (True, False):
        for b in range(3):
            tr = oracle.rollout_trace(77, b, 300, opponent=1, agent_white=white)
            env = oracle.OracleEnv(opponent=1, agent_white=white, seed=77, board=b)
            for p in range(300):
                if not env.moves():
                    assert tr["action"][p] == -1 and tr["reason"][p] == 4
                    env.reset()
                    continue
                a = env.pick()
                rc, rw, dn, why = env.step(a)
                assert tr["action"][p] == a and tr["reward"][p] == rw
                if rc == 1:
                    why, dn = 5, 1
                assert tr["done"][p] == dn and tr["reason"][p] == why
                if dn:
                    env.reset()


def test_host_opponent_mode_vs_reference_traces():
    """The device code (gc_env.h env_step_vs / env_open_vs, host build) on the same traces."""
    from core_host import corehost as H
    from gym_chess_amd import codec as C

    n = 0
    for t in load_golden("v2_opp_traces.json.gz"):
        env = H.HostEnv(_init(t), opponent=1, agent_white=t["color"] == "WHITE", seed=t["seed"], board=t["board"])
        for s in t["steps"]:
            if s["kind"] == "reset":
                env.reset()
                assert env.draw == s["draw"]
                continue
            a = env.pick()
            assert a == s["action"]
            rc, rw, dn, why = env.step(a)
            if s["kind"] == "error":
                assert rc == 1
                continue
            if s["kind"] == "opp_no_move":
                assert why == 9
                continue
            assert rc == 0 and rw == s["reward"] and bool(dn) == s["done"], s
            b, m = env.state()
            assert C.board_to_text(b) == s["board"] and list(m[:7]) == s["meta"] and m[7] == s["move_count"], s
            assert len(env.moves()) == s["n_moves"] and env.draw == s["draw"]
            n += 1
    assert n > 3000


@pytest.mark.parametrize("white", [True, False])
def test_host_opponent_rollouts_vs_oracle(oracle, white):
    from core_host import corehost as H

    sparse = np.zeros(64, dtype=np.int8)
    sparse[[60, 56, 51, 4, 12, 7]] = [1, 3, 2, -1, -6, -3]
    for init in (oracle.DEFAULT_BOARD, sparse):
        for b in range(24):
            ref = oracle.rollout_trace(0x77, b, 700, init=init, opponent=1, agent_white=white)
            got = H.rollout_trace(0x77, b, 700, init, opponent=1, agent_white=white)
            for k in ("action", "reward", "done", "reason", "final_board", "final_meta", "stats"):
                assert (np.asarray(got[k]) == np.asarray(ref[k])).all(), (b, k)


# ------------------------------------------------------------------------------- GPU
def _expected_plies(steps):
    """reference trace entries -> one expected record per device ply of the self-play driver"""
    out, j = [], 0
    while j < len(steps):
        s = steps[j]
        if s["kind"] == "reset":  # empty move list: the driver resets without a step
            out.append(dict(action=None, reason=4))
            j += 1
            continue
        rec = dict(action=s["action"], kind=s["kind"], s=s)
        j += 1
        if j < len(steps) and steps[j]["kind"] == "reset" and s["kind"] in ("error", "opp_no_move") or (
                s["kind"] == "step" and s["done"]):
            j += 1  # the reset that follows a terminal step happens inside the same device ply
        out.append(rec)
    return out


@pytest.mark.gpu
def test_gpu_opponent_mode_vs_reference_traces():
    from gym_chess_amd import codec as C
    from gym_chess_amd.env import BatchedChessEnv

    traces = load_golden("v2_opp_traces.json.gz")
    checked = 0
    for color in ("WHITE", "BLACK"):
        for sparse in (False, True):
            group = [t for t in traces if t["color"] == color and (t["initial_board"] is not None) == sparse]
            if not group:
                continue
            ib = None if not sparse else C.text_to_board(group[0]["initial_board"])
            seed = group[0]["seed"]
            nb = max(t["board"] for t in group) + 1
            env = BatchedChessEnv(nb, device=0, seed=seed, initial_board=ib, opponent="random", player_color=color)
            plans = {t["board"]: _expected_plies(t["steps"]) for t in group}
            for p in range(max(len(v) for v in plans.values())):
                act = env.outputs()["next_action"].copy()
                env.step_random(1)
                out = env.outputs()
                b, m = env.boards()
                for bid, plan in plans.items():
                    if p >= len(plan):
                        continue
                    e = plan[p]
                    if e["action"] is None:
                        assert act[bid] == 0xFFFF and out["reason"][bid] == 4, (bid, p)
                        continue
                    assert act[bid] == e["action"], (bid, p)
                    if e["kind"] == "error":
                        assert out["reason"][bid] == 5
                        continue
                    if e["kind"] == "opp_no_move":
                        assert out["reason"][bid] == 9
                        continue
                    s = e["s"]
                    assert out["reward"][bid] == s["reward"] and bool(out["done"][bid]) == s["done"], (bid, p, s)
                    if not s["done"]:
                        assert C.board_to_text(b[bid]) == s["board"], (bid, p)
                        assert list(m[bid, :7]) == s["meta"] and m[bid, 7] == s["move_count"], (bid, p)
                    checked += 1
            env.close()
    assert checked > 3000


@pytest.mark.gpu
@pytest.mark.parametrize("color", ["WHITE", "BLACK"])
def test_gpu_opponent_rollouts_vs_oracle(oracle, color):
    from gym_chess_amd.env import BatchedChessEnv

    n, plies = 256, 600
    env = BatchedChessEnv(n, device=0, seed=0x5151, opponent="random", player_color=color)
    st, tr = env.rollout(plies, trace=True)
    b, m = env.boards()
    tot = np.zeros(8, dtype=np.uint64)
    for i in range(n):
        ref = oracle.rollout_trace(0x5151, i, plies, opponent=1, agent_white=color == "WHITE")
        for k in ("action", "reward", "done", "reason"):
            assert (tr[k][:, i] == ref[k]).all(), (i, k)
        assert (b[i] == ref["final_board"]).all() and (m[i] == ref["final_meta"]).all(), i
        tot += ref["stats"]
    assert (st == tot).all()
    # the one-ply kernel path gives the same trajectories
    env2 = BatchedChessEnv(n, device=0, seed=0x5151, opponent="random", player_color=color)
    env2.step_random(plies)
    b2, m2 = env2.boards()
    assert (b2 == b).all() and (m2 == m).all()


@pytest.mark.gpu
@pytest.mark.parametrize("color", ["WHITE", "BLACK"])
@pytest.mark.parametrize("streams,sparse", [(1, False), (2, False), (2, True)])
def test_gpu_opponent_paired_step_vs_oracle(oracle, color, streams, sparse):
    """The paired opponent kernels (k_env_step2<false, 1|2>: agent ply, reply, BLACK opening,
    one pair_half each) ply by ply against the oracle's trace: every step's reward / done /
    reason and next action, the final boards; then the fused paired rollout's stats.  200
    boards: the last workgroup is partly dead lanes."""
    from gym_chess_amd.env import BatchedChessEnv

    n, plies, seed = 200, 500, 0x7A7A
    init = oracle.DEFAULT_BOARD
    if sparse:  # 6 pieces: short games, many resets and BLACK openings
        init = np.zeros(64, dtype=np.int8)
        init[[60, 56, 51, 4, 12, 7]] = [1, 3, 2, -1, -6, -3]
    kw = dict(opponent=1, agent_white=color == "WHITE", init=init)
    refs = [oracle.rollout_trace(seed, i, plies + 1, **kw) for i in range(n)]
    exp = {k: np.stack([r[k] for r in refs], axis=1) for k in ("action", "reward", "done", "reason")}
    ib = init if sparse else None
    env = BatchedChessEnv(n, device=0, seed=seed, initial_board=ib, opponent="random", player_color=color)
    assert env.paired()
    env.set_streams(streams)
    for p in range(plies):
        assert (env.outputs()["next_action"].astype(np.int64) == (exp["action"][p].astype(np.int64) & 0xFFFF)).all(), p
        env.step_random(1)
        out = env.outputs()
        for k in ("reward", "done", "reason"):
            assert (out[k].astype(np.int64) == exp[k][p].astype(np.int64)).all(), (p, k)
    env.close()

    fused = BatchedChessEnv(n, device=0, seed=seed, initial_board=ib, opponent="random", player_color=color)
    st, _ = fused.rollout(plies)
    b, m = fused.boards()
    tot = np.zeros(8, dtype=np.uint64)
    for i in range(n):
        ref = oracle.rollout_trace(seed, i, plies, **kw)
        assert (b[i] == ref["final_board"]).all() and (m[i] == ref["final_meta"]).all(), i
        tot += ref["stats"]
    assert (st == tot).all()
    fused.close()


@pytest.mark.gpu
@pytest.mark.parametrize("color", ["WHITE", "BLACK"])
def test_gpu_opponent_external_actions_vs_oracle_env(oracle, color):
    """step(actions) with the opponent replying on the device, against OracleEnv(opponent=1);
    every 7th action is random (mostly invalid: -10, state unchanged)."""
    from gym_chess_amd.env import BatchedChessEnv

    n = 48
    env = BatchedChessEnv(n, device=0, seed=99, opponent="random", player_color=color)
    refs = [oracle.OracleEnv(opponent=1, agent_white=color == "WHITE", seed=99, board=i) for i in range(n)]
    for r in refs:
        r.pick()  # the device env pre-picks a policy action at reset (same Philox stream)
    rng = np.random.RandomState(3)
    for ply in range(250):
        acts = np.zeros(n, dtype=np.int64)
        for i, r in enumerate(refs):
            mv = r.moves()
            acts[i] = rng.randint(0, 4101) if (ply % 7 == 6 or not mv) else mv[rng.randint(len(mv))]
        rw, dn, why = env.step(acts)
        b, m = env.boards()
        for i, r in enumerate(refs):
            rc, rr, rd, rq = r.step(int(acts[i]))
            if rc == 1:
                assert why[i] == 5
            else:
                assert (rw[i], bool(dn[i]), why[i]) == (rr, bool(rd), rq), (ply, i)
                rb, rm = r.state()
                assert (b[i] == rb).all() and (m[i] == rm).all(), (ply, i)
        done = np.array([bool(dn[i]) or why[i] == 5 for i in range(n)])
        if done.any():
            env.reset(done.astype(np.uint8))
            for i in np.nonzero(done)[0]:
                refs[i].reset()
                refs[i].pick()
