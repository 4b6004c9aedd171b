"""Bit-exact checkpoint / resume of the batched env (gc_env_save / gc_env_load).

The reference env's history lives in ChessEnvV2.saved_boards (chess_v2.py:192, 404-407)
next to the state dict (301-323); a restore that dropped it would restart every 3-fold
count.  Here: run, save, run on, reload (into the same env and into a fresh one), run the
same plies again -> identical per-ply outputs and states; and the restored env's plies ==
the oracle's uninterrupted trajectory (whose saved_boards is the restated history)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _plies(env, k):
    out = []
    for _ in range(k):
        env.step_random(1)
        o = env.outputs()
        out.append((o["reward"].copy(), o["done"].copy(), o["reason"].copy(), o["next_action"].copy()))
    return out


def _same(a, b):
    return all(all((x == y).all() for x, y in zip(p, q)) for p, q in zip(a, b))


@pytest.mark.parametrize("kw", [dict(), dict(opponent="random"), dict(opponent="random", player_color="BLACK"),
                                dict(rules="fide")], ids=["none", "random", "random_black", "fide"])
def test_save_run_reload_rerun(kw):
    from gym_chess_amd.env import BatchedChessEnv

    n, seed = 1000, 2024
    env = BatchedChessEnv(n, device=0, seed=seed, **kw)
    env.step_random(150)
    blob = env.checkpoint()
    b0, m0 = env.boards()
    first = _plies(env, 300)
    bf, mf = env.boards()
    env.load(blob)
    b1, m1 = env.boards()
    assert (b0 == b1).all() and (m0 == m1).all()
    again = _plies(env, 300)
    assert _same(first, again)
    b2, m2 = env.boards()
    assert (bf == b2).all() and (mf == m2).all()
    # a fresh env built with the same arguments
    fresh = BatchedChessEnv(n, device=0, seed=seed, **kw)
    fresh.load(blob)
    assert _same(first, _plies(fresh, 300))
    b3, m3 = fresh.boards()
    assert (bf == b3).all() and (mf == m3).all()
    env.close()
    fresh.close()


def test_restored_env_continues_the_oracle_trajectory(oracle):
    """Boards with live 3-fold windows at the save point: the restored env's plies 150..449 ==
    the oracle's uninterrupted 450-ply trajectories (repetitions included)."""
    from gym_chess_amd.env import BatchedChessEnv

    n, seed, cut, tot = 256, 4711, 150, 450
    env = BatchedChessEnv(n, device=0, seed=seed)
    env.step_random(cut)
    assert env.window_sum() > 0  # something to carry over
    blob = env.checkpoint()
    env.close()
    fresh = BatchedChessEnv(n, device=0, seed=seed)
    fresh.step_random(37)  # the fresh env's own windows and streams must not leak through
    fresh.load(blob)
    got = _plies(fresh, tot - cut)
    refs = [oracle.rollout_trace(seed, i, tot + 1) for i in range(n)]
    for p in range(tot - cut):
        rw, dn, why, nxt = got[p]
        want_r = np.array([r["reward"][cut + p] for r in refs])
        want_q = np.array([r["reason"][cut + p] for r in refs])
        want_a = np.array([r["action"][cut + p + 1] for r in refs])
        assert (rw == want_r).all() and (why == want_q).all(), p
        assert (nxt == np.where(want_a < 0, 0xFFFF, want_a).astype(np.uint16)).all(), p


def test_knight_shuffle_repetition_survives_restore():
    """Nf3 Nf6 Ng1 Ng8 Nf3 Nf6 Ng1 Ng8 Nf3: the reference env ends on ply 9 (3-fold on the
    pre-move board, chess_v2.py:404-407).  Saved after ply 4 and restored into a fresh env,
    the game still ends on ply 9; the same boards set through set_states (no history) do not."""
    from gym_chess_amd.env import BatchedChessEnv

    seq = [62 * 64 + 45, 6 * 64 + 21, 45 * 64 + 62, 21 * 64 + 6] * 2 + [62 * 64 + 45]  # g1f3 g8f6 f3g1 f6g8 ...
    n = 8
    env = BatchedChessEnv(n, device=0, seed=5)
    for a in seq[:4]:
        rw, dn, why = env.step(np.full(n, a))
        assert not dn.any()
    blob = env.checkpoint()
    b, m = env.boards()
    fresh = BatchedChessEnv(n, device=0, seed=5)
    fresh.load(blob)
    nohist = BatchedChessEnv(n, device=0, seed=5)
    nohist.set_states(b, m)
    for k, a in enumerate(seq[4:]):
        rw, dn, why = fresh.step(np.full(n, a))
        rw2, dn2, why2 = nohist.step(np.full(n, a))
        last = k == len(seq) - 5
        assert dn.all() == last and (why == (2 if last else 0)).all(), (k, why)
        assert not dn2.any()


def test_load_rejects_mismatched_env():
    from gym_chess_amd._lib import GymChessError
    from gym_chess_amd.env import BatchedChessEnv

    env = BatchedChessEnv(64, device=0, seed=1)
    blob = env.checkpoint()
    for kw in (dict(num_boards=65, seed=1), dict(num_boards=64, seed=2), dict(num_boards=64, seed=1, rules="fide"),
               dict(num_boards=64, seed=1, opponent="random")):
        other = BatchedChessEnv(device=0, **kw)
        with pytest.raises(GymChessError):
            other.load(blob)
        other.close()
    with pytest.raises(GymChessError):
        env.load(blob[:-1])
    with pytest.raises(GymChessError):
        env.load(b"x" * len(blob))
