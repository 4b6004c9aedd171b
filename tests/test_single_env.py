"""Single-board ChessEnv (gym_chess_amd.single: the ChessEnvV2 surface, its bookkeeping in
one device launch per step) against the reference ChessEnvV2's own recorded traces
(tests/golden/v2_env_traces.json.gz, written by make_golden.py from the reference env):
opponent "none" and "random" (numpy's global generator, so the seeded driver below replays
the reference's games move for move), invalid actions, 3-fold, kingless play.  CPU: over the
oracle's restatement of the same ops (tests/oracle_engine.OracleBoard); GPU: on the device.
"""
import numpy as np
import pytest

from conftest import load_golden


def _replay(make_env, t):
    from gym_chess_amd import codec as C

    ib = None if t.get("initial_board") is None else C.text_to_board(t["initial_board"]).reshape(8, 8)
    kw = dict(log=False)
    if ib is not None:
        kw["initial_board"] = ib
    if t.get("scripted"):
        env = make_env(opponent="none", **kw)
        for a, s in zip(t["actions"], t["steps"]):
            _check(env, env.step(int(a)), s)
        return len(t["steps"])
    np.random.seed(t["seed"])  # the same generator calls as make_golden.trace_env
    env = make_env(opponent=t["opponent"], **kw)
    rng = np.random.RandomState(t["seed"] + 7)
    steps = t["steps"]
    j, i, every = 0, 0, t["invalid_every"]
    while j < len(steps):
        moves = env.possible_moves
        if not moves:
            assert steps[j]["kind"] == "reset"
            env.reset()
            j += 1
            i += 1
            continue
        if every and i % every == every - 1:
            action = int(rng.randint(0, 4100))
        else:
            action = env.move_to_action(moves[np.random.choice(np.arange(len(moves)))])
        s = steps[j]
        assert s.get("action") == action, (j, s, action)
        try:
            out = env.step(action)
        except SystemError:
            assert s["kind"] == "error"
            env.reset()
            j += 1
            i += 1
            continue
        _check(env, out, s)
        j += 1
        i += 1
        if out[2]:
            assert steps[j]["kind"] == "reset"
            env.reset()
            j += 1
    return j


def _check(env, out, s):
    from gym_chess_amd import codec as C

    state, reward, done, info = out
    assert s["kind"] == "step"
    assert reward == s["reward"] and bool(done) == s["done"], s
    assert C.board_to_text(np.asarray(state["board"]).reshape(64)) == s["board"]
    assert info["move_count"] == s["move_count"] and len(env.possible_moves) == s["n_moves"]
    if "meta" in s:
        got = [int(env.current_player == "WHITE"), int(state["white_king_castle_is_possible"]),
               int(state["white_queen_castle_is_possible"]), int(state["black_king_castle_is_possible"]),
               int(state["black_queen_castle_is_possible"]), int(bool(state["white_king_is_checked"])),
               int(bool(state["black_king_is_checked"]))]
        assert got == s["meta"], s


def test_single_env_traces_on_oracle_engine():
    from gym_chess_amd.single import ChessEnv
    from oracle_engine import OracleBoard, OracleChessEngine

    eng = OracleChessEngine()
    n = 0
    for t in load_golden("v2_env_traces.json.gz"):
        n += _replay(lambda **kw: ChessEnv(backend=OracleBoard(kw.get("initial_board")), engine=eng, **kw), t)
    assert n > 3000


def test_single_env_black_player_and_errors():
    from gym_chess_amd import codec as C
    from gym_chess_amd.single import ChessEnv
    from oracle_engine import OracleBoard

    np.random.seed(5)
    env = ChessEnv(player_color=C.BLACK, opponent="random", log=False, backend=OracleBoard())
    assert env.current_player == C.BLACK and env.move_count == 1
    assert sum(1 for row in env.board for v in row if v > 0) == 16
    acts = env.possible_actions
    assert len(acts) == 20
    with pytest.raises(AssertionError):
        env.step(4101)
    _, r, d, _ = env.step(0)  # a8a8: not legal -> -10, state unchanged
    assert r == -10 and not d and env.move_count == 1
    env2 = ChessEnv(opponent="none", log=False, backend=OracleBoard())
    assert env2.render(mode="string").count("\n") == 11
    with pytest.raises(ValueError):
        ChessEnv(opponent="bogus", log=False, backend=OracleBoard())


@pytest.mark.gpu
def test_single_env_traces_on_gpu_engine():
    from gym_chess_amd.engine import ChessEngine
    from gym_chess_amd.single import ChessEnv

    eng = ChessEngine(0)
    n = 0
    for t in load_golden("v2_env_traces.json.gz"):
        n += _replay(lambda **kw: ChessEnv(engine=eng, **kw), t)
    assert n > 3000


@pytest.mark.gpu
def test_single_env_device_extras():
    """BLACK agent with a callable opponent, the live window readout (saved_boards), logging,
    state assignment, and the stateless helpers on the device engine."""
    import contextlib
    import io

    from gym_chess_amd import codec as C
    from gym_chess_amd.single import ChessEnv

    def knight_move(e):  # reversible moves only: the window keeps growing
        return next(m for m in e.possible_moves if not isinstance(m, str) and abs(e.board[m[0][0]][m[0][1]]) == 5)

    np.random.seed(11)
    env = ChessEnv(player_color=C.BLACK, opponent=knight_move, log=False)
    assert env.current_player == C.BLACK and env.move_count == 1
    for _ in range(6):
        env.step(env.move_to_action(knight_move(env)))
    sb = env.device_window()
    assert len(sb) >= 3 and sum(sb.values()) >= 6 and all(1 <= v <= 2 for v in sb.values()), sb.values()
    # saved_boards: every pre-move board since reset (the opening + 6 x (agent, opponent))
    assert sum(env.saved_boards.values()) == 13 and all(len(k) == 64 for k in env.saved_boards)
    env = ChessEnv(opponent="none", log=True)
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        env.step(env.possible_actions[0])
    assert ">>>>>>>>>>" in buf.getvalue() and "WHITE" in buf.getvalue()
    st = env.state
    st["board"] = C.DEFAULT_BOARD
    before = dict(env.saved_boards)
    env.state = st
    # the setter (chess_v2.py:315-323) keeps saved_boards, the side to move and the stale list
    assert env.board == np.asarray(C.DEFAULT_BOARD).reshape(8, 8).tolist() and env.saved_boards == before
    assert env.current_player == C.BLACK and len(before) == 1
    assert len(env.get_possible_moves(state=env.state, player=C.WHITE)) == 20


def _replay_setter(env, t):
    """tests/golden/v2_setter_traces.json.gz (the reference ChessEnvV2 with state assignments
    between steps): every step's outputs and the whole saved_boards dict"""
    from gym_chess_amd import codec as C

    n = 0
    for o in t["ops"]:
        if o["kind"] == "reset":
            env.reset()
        elif o["kind"] == "set":
            b = C.text_to_board(o["board"]).reshape(8, 8)
            keys = ("white_king_castle_is_possible", "white_queen_castle_is_possible", "black_king_castle_is_possible",
                    "black_queen_castle_is_possible", "white_king_is_checked", "black_king_is_checked")
            st = dict(board=b.tolist(), current_player="BLACK", **{k: bool(f) for k, f in zip(keys, o["flags"])})
            env.state = st  # (current_player ignored by the setter, chess_v2.py:315-323)
        elif o["kind"] == "error":
            with pytest.raises(SystemError):
                env.step(o["action"])
            env.reset()
        else:
            _check(env, env.step(o["action"]), o)
            got = sorted([k, v] for k, v in env.saved_boards.items())
            assert got == o["saved"], (n, len(got), len(o["saved"]))
            n += 1
    return n


def test_single_env_state_setter_on_oracle_engine():
    """ADVICE r03 / VERDICT r03 #9: the state setter changes the board and flags only (the side
    to move, move_count, done and the stale possible_moves stay) and saved_boards is the
    reference's whole-history dict -- replayed against the reference env's own traces."""
    from gym_chess_amd.single import ChessEnv
    from oracle_engine import OracleBoard, OracleChessEngine

    eng = OracleChessEngine()
    n = 0
    for t in load_golden("v2_setter_traces.json.gz"):
        n += _replay_setter(ChessEnv(opponent="none", log=False, backend=OracleBoard(), engine=eng), t)
    assert n > 1000


@pytest.mark.gpu
def test_single_env_state_setter_on_gpu():
    from gym_chess_amd.engine import ChessEngine
    from gym_chess_amd.single import ChessEnv

    eng = ChessEngine(0)
    n = 0
    for t in load_golden("v2_setter_traces.json.gz"):
        env = ChessEnv(opponent="none", log=False, engine=eng)
        n += _replay_setter(env, t)
        env.close()
    assert n > 1000


def test_state_setter_missing_flags_default_false():
    """a state dict without some flags: False (the reference stores None, which its engine then
    rejects on the next call)"""
    from gym_chess_amd import codec as C
    from gym_chess_amd.single import ChessEnv
    from oracle_engine import OracleBoard

    env = ChessEnv(opponent="none", log=False, backend=OracleBoard())
    env.state = dict(board=np.asarray(C.DEFAULT_BOARD).reshape(8, 8).tolist())
    assert env.white_king_castle_is_possible is False and env.black_king_is_checked is False
    assert len(env.possible_moves) == 20  # stale: the list of the board before (the same board here)


@pytest.mark.gpu
def test_single_env_server_idle_exit_and_restart():
    """The single-board server (k_single_server: one resident wave serving requests through a
    host-mapped mailbox) exits after 50 ms without a request and is started again by the next
    one; ops that need the stream (the window readout) stop it first.  The trajectory equals the
    oracle backend's, step for step, across the restarts."""
    import time

    from gym_chess_amd.single import ChessEnv
    from oracle_engine import OracleBoard

    dev = ChessEnv(opponent="none", log=False)
    ref = ChessEnv(opponent="none", log=False, backend=OracleBoard())
    rng = np.random.RandomState(3)
    for t in range(160):
        acts = ref.possible_actions
        if not acts:
            dev.reset(); ref.reset()
            continue
        a = int(acts[rng.randint(len(acts))])
        o1, o2 = dev.step(a), ref.step(a)
        assert o1[1:3] == o2[1:3] and o1[0]["board"] == o2[0]["board"], t
        assert dev.possible_actions == ref.possible_actions and dev.saved_boards == ref.saved_boards, t
        if t % 40 == 17:
            time.sleep(0.12)  # the server times out; the next step starts it again
        if t % 40 == 29:
            dev.device_window()  # a stream op: the server is stopped first
        if o1[2]:
            dev.reset(); ref.reset()
    dev.close()


@pytest.mark.gpu
def test_resident_servers_stopped_at_process_exit():
    """A process that ends right after its last server call (no close / destroy) stops the
    resident waves (engine server, single-board server) in the library's exit handler."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from gym_chess_amd import codec as C\n"
            "from gym_chess_amd.engine import ChessEngine\n"
            "from gym_chess_amd.single import ChessEnv\n"
            "e = ChessEngine(0)\n"
            "st = dict(board=C.DEFAULT_BOARD, current_player='WHITE', white_king_castle_is_possible=True,"
            " white_queen_castle_is_possible=True, black_king_castle_is_possible=True, black_queen_castle_is_possible=True)\n"
            "assert len(e.get_possible_moves(st, 'WHITE')) == 20\n"
            "env = ChessEnv(opponent='none', log=False)\n"
            "env.step(env.possible_actions[0])\n" % os.path.join(root, "gym-chess_amd"))
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120,
                         env=dict(os.environ, GC_SRV_EXIT_LOG="1"))
    assert out.returncode == 0, out.stderr[-2000:]
    assert "did not answer" not in out.stderr, out.stderr[-2000:]


@pytest.mark.gpu
def test_many_servers_round_robin_no_stall():
    """seven single-board envs stepped round-robin (a vector env), each step
    interleaved with a ChessEngine one-position call and a batched env's launched ply.  Every
    one of them would keep a resident server, and the process has more streams than hardware
    queues, so a server queued behind another's waited for it to idle out (~50 ms).  One
    resident server per device (the others stopped on demand): no call stalls, and every
    trajectory equals its oracle twin's."""
    import time

    from gym_chess_amd import codec as C
    from gym_chess_amd.engine import ChessEngine
    from gym_chess_amd.env import BatchedChessEnv
    from gym_chess_amd.single import ChessEnv
    from oracle_engine import OracleBoard

    k = 7
    devs = [ChessEnv(opponent="none", log=False) for _ in range(k)]
    refs = [ChessEnv(opponent="none", log=False, backend=OracleBoard()) for _ in range(k)]
    eng = ChessEngine(0)
    batched = BatchedChessEnv(256, device=0, seed=5)
    st = dict(board=C.DEFAULT_BOARD, current_player="WHITE", white_king_castle_is_possible=True,
              white_queen_castle_is_possible=True, black_king_castle_is_possible=True,
              black_queen_castle_is_possible=True)
    rng = np.random.RandomState(11)
    times = []
    for t in range(30):
        for j in range(k):
            acts = refs[j].possible_actions
            if not acts:
                devs[j].reset(); refs[j].reset()
                continue
            a = int(acts[rng.randint(len(acts))])
            t0 = time.perf_counter()
            o1 = devs[j].step(a)
            assert len(eng.get_possible_moves(st, "WHITE")) == 20
            times.append(time.perf_counter() - t0)
            o2 = refs[j].step(a)
            assert o1[1:3] == o2[1:3] and o1[0]["board"] == o2[0]["board"], (t, j)
            assert devs[j].possible_actions == refs[j].possible_actions, (t, j)
            if o1[2]:
                devs[j].reset(); refs[j].reset()
        t0 = time.perf_counter()
        batched.step_random(1)
        batched.synchronize()
        times.append(time.perf_counter() - t0)
    times = np.array(times) * 1e3
    for e in devs:
        e.close()
    batched.close()
    # a stall is one SRV_IDLE_MS (50 ms); a server switch costs a stop and a launch (~0.1 ms)
    assert np.percentile(times, 99) < 10.0 and times.mean() < 3.0, (times.mean(), np.percentile(times, 99), times.max())
