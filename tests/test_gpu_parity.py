"""GPU parity: the HIP kernels (through the C-ABI) vs the oracle and the golden fixtures.

Bar: bit-exact (integer work) -- ordered move lists, next states, rewards, check flags,
perft counts, step() rewards/done/reasons and whole random-self-play trajectories.
"""
import numpy as np
import pytest

from conftest import load_golden, random_positions

pytestmark = pytest.mark.gpu


def _text_board(t):
    from gym_chess_amd import codec as C

    return C.text_to_board(t)


# ------------------------------------------------------------------ engine: move lists
def test_v1_games_ordered_lists(engine):
    """1888 positions along seeded v1 reference games (D4-transformed, D-filtered)."""
    games = load_golden("v1_games.json.gz")
    plies = [p for g in games for p in g["plies"]]
    b = np.stack([_text_board(p["board"]) for p in plies])
    m = np.zeros((len(plies), 8), dtype=np.uint8)
    m[:, 0] = [p["white"] for p in plies]
    m[:, 1:5] = [p["rights"] for p in plies]
    out, cnt = engine.possible_moves(b, m, m[:, 0])
    for i, p in enumerate(plies):
        assert [int(x) for x in out[i, : cnt[i]]] == p["moves"], f"ply {i}"
    # next boards and rewards of the chosen actions
    acts = np.array([p["action"] for p in plies], dtype=np.uint16)
    nb, nm, rw, st = engine.next_state(b, m, m[:, 0], acts)
    assert (st == 0).all()
    for i, p in enumerate(plies):
        assert (nb[i] == _text_board(p["next_board"])).all(), f"ply {i}"
        assert rw[i] == p["reward"]


def test_v2_known_answers(engine):
    """Every engine call the reference's own v2 tests made (their asserts passed)."""
    cases = load_golden("v2_known_answers.json")
    n = 0
    for case in cases:
        for c in case["calls"]:
            b = _text_board(c["board"])[None]
            m = np.zeros((1, 8), dtype=np.uint8)
            m[0, :5] = c["meta"]
            if c["op"] == "get_possible_moves":
                out, cnt = engine.possible_moves(b, m, c["white"], attack=c["attack"])
                assert [int(x) for x in out[0, : cnt[0]]] == c["out"], (case["test"], c)
            elif c["op"] == "get_castle_moves":
                out, cnt = engine.castle_moves(b, m, c["white"])
                assert [int(x) for x in out[0, : cnt[0]]] == c["out"], case["test"]
            elif c["op"] == "update_state":
                ob, om = engine.update_state(b, m)
                assert list(om[0, :7]) == c["out_meta"], case["test"]
            elif c["op"] == "next_state":
                ob, om, rw, st = engine.next_state(b, m, c["white"], c["action"])
                assert (ob[0] == _text_board(c["out_board"])).all()
                assert list(om[0, :7]) == c["out_meta"] and rw[0] == c["reward"]
                assert bool(st[0] == 1) == c["both_checked"]
            n += 1
    assert n >= 60


@pytest.mark.parametrize("seed", [11, 12, 13])
def test_random_positions_vs_oracle(engine, oracle, seed):
    """Fuzz: legal + attack-mode lists, castle lists, update_state, next_state of every
    legal move and of arbitrary (also illegal / wrong-player) moves."""
    boards, metas = random_positions(400, seed)
    for attack in (False, True):
        for white in (0, 1):
            out, cnt = engine.possible_moves(boards, metas, white, attack=attack)
            for i in range(len(boards)):
                ref = oracle.get_possible_moves(boards[i], metas[i], white, attack)
                assert [int(x) for x in out[i, : cnt[i]]] == ref, (i, attack, white)
    cm, cc = engine.castle_moves(boards, metas, metas[:, 0])
    ob, om = engine.update_state(boards, metas)
    rng = np.random.RandomState(seed)
    acts = np.zeros(len(boards), dtype=np.uint16)
    players = rng.randint(2, size=len(boards)).astype(np.uint8)
    for i in range(len(boards)):
        assert [int(x) for x in cm[i, : cc[i]]] == oracle.get_castle_moves(boards[i], metas[i], metas[i, 0])
        rb, rm = oracle.update_state(boards[i], metas[i])
        assert (ob[i] == rb).all() and list(om[i, :7]) == list(rm[:7]), i
        occupied = np.nonzero(boards[i])[0]
        if rng.rand() < 0.2:
            acts[i] = 4096 + rng.randint(4)
        else:
            acts[i] = int(rng.choice(occupied)) * 64 + rng.randint(64)
    nb, nm, rw, st = engine.next_state(boards, metas, players, acts)
    for i in range(len(boards)):
        rc, rb, rm, rr = oracle.next_state(boards[i], metas[i], players[i], int(acts[i]))
        assert st[i] == rc, i
        if rc in (0, 1):
            assert (nb[i] == rb).all() and list(nm[i, :7]) == list(rm[:7]) and rw[i] == rr, i


def test_one_position_calls_vs_oracle(engine, oracle):
    """The engine server (k_engine_server: every n = 1 call under the reference rules, the
    drop-in ChessEngine's shape): legal and attack-mode lists for both players, castle
    lists, update_state and next_state of arbitrary moves, one position per call."""
    boards, metas = random_positions(150, 31)
    rng = np.random.RandomState(31)
    for i in range(len(boards)):
        b, m = boards[i:i + 1], metas[i:i + 1]
        for attack in (False, True):
            for white in (0, 1):
                out, cnt = engine.possible_moves(b, m, white, attack=attack)
                assert [int(x) for x in out[0, : cnt[0]]] == oracle.get_possible_moves(b[0], m[0], white, attack), i
        cm, cc = engine.castle_moves(b, m, m[:, 0])
        assert [int(x) for x in cm[0, : cc[0]]] == oracle.get_castle_moves(b[0], m[0], m[0, 0]), i
        ob, om = engine.update_state(b, m)
        rb, rm = oracle.update_state(b[0], m[0])
        assert (ob[0] == rb).all() and list(om[0, :7]) == list(rm[:7]), i
        occupied = np.nonzero(b[0])[0]
        a = 4096 + rng.randint(4) if rng.rand() < 0.2 else int(rng.choice(occupied)) * 64 + rng.randint(64)
        p = rng.randint(2)
        nb, nm, rw, st = engine.next_state(b, m, p, a)
        rc, rb, rm, rr = oracle.next_state(b[0], m[0], p, a)
        assert st[0] == rc, i
        if rc in (0, 1):
            assert (nb[0] == rb).all() and list(nm[0, :7]) == list(rm[:7]) and rw[0] == rr, i


def test_one_position_calls_from_two_threads(engine, oracle):
    """ctypes releases the GIL: two threads calling one engine at once (the server's mailbox
    and the staging buffers are the engine's) get every list right."""
    import threading

    boards, metas = random_positions(80, 41)
    refs = [oracle.get_possible_moves(boards[i], metas[i], int(metas[i, 0]), False) for i in range(80)]
    errors = []

    def work(lo, hi):
        for _ in range(5):
            for i in range(lo, hi):
                out, cnt = engine.possible_moves(boards[i:i + 1], metas[i:i + 1], int(metas[i, 0]))
                if [int(x) for x in out[0, : cnt[0]]] != refs[i]:
                    errors.append(i)

    ts = [threading.Thread(target=work, args=(0, 40)), threading.Thread(target=work, args=(40, 80))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors[:8]


def test_chess_engine_dict_calls_from_two_threads(oracle):
    """the drop-in ChessEngine reuses its output buffers across calls; two threads
    sharing one instance (ctypes releases the GIL) must each get their own lists and next
    states -- the lock covers the C call and the conversion to Python objects."""
    import threading

    from gym_chess_amd import codec as C
    from gym_chess_amd.engine import ChessEngine

    eng = ChessEngine(0)
    boards, metas = random_positions(60, 43, weird=False)
    states, want_lists, want_next = [], [], []
    for i in range(60):
        b, m = boards[i], metas[i]
        st = C.arrays_to_dict(b, m)
        white = int(m[0])
        lst = oracle.get_possible_moves(b, m, white)
        states.append((st, "WHITE" if white else "BLACK"))
        want_lists.append(C.actions_to_strs(np.array(lst, dtype=np.uint16)))
        if lst:
            rc, nb, nm, rw = oracle.next_state(b, m, white, lst[0])
            want_next.append((C.action_to_str(lst[0]), nb, rw) if rc == 0 else None)
        else:
            want_next.append(None)
    errors = []

    def work(lo, hi):
        for _ in range(4):
            for i in range(lo, hi):
                st, pl = states[i]
                if eng.get_possible_moves(st, pl) != want_lists[i]:
                    errors.append(("list", i))
                if want_next[i] is not None:
                    mv, nb, rw = want_next[i]
                    d, r = eng.next_state(st, pl, mv)
                    if r != rw or list(np.asarray(d["board"]).reshape(64)) != list(nb):
                        errors.append(("next", i))

    ts = [threading.Thread(target=work, args=(0, 30)), threading.Thread(target=work, args=(30, 60))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors[:8]


@pytest.mark.parametrize("mirror", [False, True])
def test_two_pins_double_push_never_crosses_its_king(engine, oracle, mirror):
    """Two pins on the king's file (rook behind, queen in front): the rear pawn's Q1 double push
    must not jump the king onto the front pin's segment (tests/test_core_host.py TWO_PINS; the
    soak's board 65 486): lists one at a time and batched, perft, the policy's pick."""
    from test_core_host import _two_pins_position

    b, m = _two_pins_position(mirror)
    w = int(m[0])
    ref = oracle.get_possible_moves(b, m, w)
    out, cnt = engine.possible_moves(b[None], m[None], w)
    assert [int(x) for x in out[0, : cnt[0]]] == ref
    bb, mm = np.repeat(b[None], 300, axis=0), np.repeat(m[None], 300, axis=0)
    out, cnt = engine.possible_moves(bb, mm, w)
    assert all([int(x) for x in out[i, : cnt[i]]] == ref for i in range(300))
    assert (engine.perft(bb[:2], mm[:2], 3) == oracle.perft(b, m, 3)).all()


def test_two_pins_soak_board_65486_fused_vs_oracle(oracle):
    """The soak's failing trajectory (seed 1000, board 65 486, the divergence at ply 4 591)
    through the headline kernel: every ply of that board == the oracle's."""
    from gym_chess_amd.env import BatchedChessEnv

    env = BatchedChessEnv(65536, device=0, seed=1000)
    tb = env.trace_buffer(4600)
    env.rollout_device(4600, tb)
    env.synchronize()
    tr = tb.fetch()
    ref = oracle.rollout_trace(1000, 65486, 4600)
    for key in ("action", "reward", "done", "reason"):
        assert (tr[key][:, 65486] == ref[key]).all(), key
    tb.close()
    env.close()


def test_next_state_every_legal_move(engine, oracle):
    boards, metas = random_positions(150, 21)
    B, M, P, A = [], [], [], []
    for i in range(len(boards)):
        w = int(metas[i, 0])
        for a in oracle.get_possible_moves(boards[i], metas[i], w):
            B.append(boards[i]); M.append(metas[i]); P.append(w); A.append(a)
    B, M = np.stack(B), np.stack(M)
    nb, nm, rw, st = engine.next_state(B, M, np.array(P, np.uint8), np.array(A, np.uint16))
    for k in range(len(A)):
        rc, rb, rm, rr = oracle.next_state(B[k], M[k], P[k], A[k])
        assert st[k] == rc and (nb[k] == rb).all() and list(nm[k, :7]) == list(rm[:7]) and rw[k] == rr, k


def test_empty_from_square_status(engine):
    b = np.zeros((1, 64), dtype=np.int8)
    b[0, 60] = 1
    m = np.zeros((1, 8), dtype=np.uint8)
    _, _, _, st = engine.next_state(b, m, 1, 36 * 64 + 28)
    assert st[0] == -1  # the reference panics: "Bad move - piece is empty !"


# ------------------------------------------------------------------ perft
def test_perft_startpos_4096_boards(engine):
    """BASELINE configs[1]: 4 096 startpos boards, perft(3) = 8 982 each (reference rules)."""
    from oracle import DEFAULT_BOARD, make_meta

    b = np.tile(DEFAULT_BOARD, (4096, 1))
    m = np.tile(make_meta(), (4096, 1))
    assert (engine.perft(b, m, 3) == 8982).all()
    golden = load_golden("perft_startpos.json")["perft"]
    got = [int(engine.perft(b[:1], m[:1], d)[0]) for d in range(1, 6)]
    assert got == [golden[str(d)] for d in range(1, 6)] == [20, 400, 8982, 200915, 5018995]


def test_perft_midgame_vs_v1(engine, oracle):
    for p in load_golden("v1_perft_midgame.json"):
        b = _text_board(p["board"])[None]
        m = np.zeros((1, 8), dtype=np.uint8)
        m[0, :5] = p["meta"]
        for d, v in p["v1_perft"].items():
            got = int(engine.perft(b, m, int(d))[0])
            if p["v1_equals_v2"]:
                assert got == v
            assert got == oracle.perft(b[0], m[0], int(d))


def test_perft_random_positions(engine, oracle):
    boards, metas = random_positions(48, 31)
    for d in (1, 2, 3):
        got = engine.perft(boards, metas, d)
        ref = oracle.perft_batch(boards, metas, d, threads=8)
        assert (got == ref).all(), d


def test_perft_sorted_subtrees_vs_oracle(engine, oracle):
    """perft(4) of 256 mid-game roots: the leaf level (~2e5 depth-2 subtrees) runs in order of
    the subtree roots' move counts (k_perft_small_perm); totals per root == the oracle's."""
    from gym_chess_amd.env import BatchedChessEnv

    env = BatchedChessEnv(256, device=0, seed=0x5EED + 4)
    env.step_random(25)
    b, m = env.boards()
    got = engine.perft(b, m, 4)
    ref = oracle.perft_batch(b, m, 4, threads=16)
    assert (got == ref).all(), np.nonzero(got != ref)[0][:4]


def test_perft_split_leaves_matches_depth3_subtrees(engine):
    """perft(5) of 200 mid-game roots: the leaf level split one more ply in chunks
    (perft_split_leaves, depth-2 subtrees sorted by move count) == the depth-3 subtrees
    (GC_PERFT_SPLIT=0), per root."""
    import os

    from gym_chess_amd.env import BatchedChessEnv

    env = BatchedChessEnv(200, device=0, seed=0x5EED + 5)
    env.step_random(21)
    b, m = env.boards()
    split = engine.perft(b, m, 5)
    os.environ["GC_PERFT_SPLIT"] = "0"
    try:
        whole = engine.perft(b, m, 5)
    finally:
        del os.environ["GC_PERFT_SPLIT"]
    assert (split == whole).all() and split.sum() > 200 * 10**6, np.nonzero(split != whole)[0][:4]


def test_perft_split_transpositions_merged_exactly(engine):
    """The split pass's transposition pass (one leaf count per distinct depth-2 root of a chunk,
    the other records adding the leader's count to their own parents) == every record counted
    (GC_PERFT_DEDUP=0), per root; the merge happened (counted < records).  The records are
    sorted by hash tag (k_dedup_keys, radix sort, k_dedup_runs_f) and the followers credited by
    their leader's leaf lane (k_perft2_val).  (The round-4 CAS table and round-5's follower pass
    were removed in round 6.)"""
    import os

    from gym_chess_amd.engine import perft_dedup_stats

    b, m = _midgame_roots(200, 21, 0x5EED + 5)
    r0, c0 = perft_dedup_stats()
    merged = engine.perft(b, m, 5)
    r1, c1 = perft_dedup_stats()
    os.environ["GC_PERFT_DEDUP"] = "0"
    try:
        every = engine.perft(b, m, 5)
    finally:
        del os.environ["GC_PERFT_DEDUP"]
    r2, c2 = perft_dedup_stats()
    assert (merged == every).all(), np.nonzero(merged != every)[0][:4]
    assert r1 - r0 == r2 - r1 == c2 - c1 > 0
    assert c1 - c0 < 0.8 * (r1 - r0), (r1 - r0, c1 - c0)


def test_perft_transpositions_over_several_chunks(engine):
    """4 096 mid-game roots: ~5e6 depth-3 subtree roots, so the split pass runs several chunks
    of 2^21 parents, each with its own transposition table; merged == every record counted,
    per root."""
    import os

    from gym_chess_amd.engine import perft_dedup_stats

    b, m = _midgame_roots(4096, 21, 0x5EED + 6)
    r0, c0 = perft_dedup_stats()
    merged = engine.perft(b, m, 5)
    r1, c1 = perft_dedup_stats()
    os.environ["GC_PERFT_DEDUP"] = "0"
    try:
        every = engine.perft(b, m, 5)
    finally:
        del os.environ["GC_PERFT_DEDUP"]
    assert (merged == every).all(), np.nonzero(merged != every)[0][:4]
    assert r1 - r0 > 2 ** 21 * 20 and c1 - c0 < 0.8 * (r1 - r0)


def _midgame_roots(n, plies, seed):
    from gym_chess_amd.env import BatchedChessEnv

    env = BatchedChessEnv(n, device=0, seed=seed)
    env.step_random(plies)
    b, m = env.boards()
    env.close()
    return b, m


def test_perft5_split_leaves_vs_oracle(engine, oracle):
    """BASELINE configs[3] path: perft(5) of 200 mid-game roots.  200 roots -> 7e3 -> 2.4e5
    nodes with 3 plies left (>= 131 072: no further expansion), so the leaf level takes the
    split pass (depth-3 subtrees split one more ply in chunks, depth-2 subtrees sorted by move
    count: perft_split_leaves) -- asserted through the path counters.  12 roots spread over
    the batch are compared with the oracle at depth 5, per root."""
    from gym_chess_amd.engine import perft_path_counts

    b, m = _midgame_roots(200, 21, 0x5EED + 5)
    c0 = perft_path_counts()
    got = engine.perft(b, m, 5)
    c1 = perft_path_counts()
    assert c1["split"] == c0["split"] + 1 and c1["sorted"] == c0["sorted"] and c1["small"] == c0["small"]
    pick = np.arange(0, 200, 25)  # 8 roots, ~3e8 nodes for the oracle
    ref = oracle.perft_by_children(b[pick], m[pick], 5, threads=16)
    assert (got[pick] == ref).all(), (pick, got[pick], ref)
    assert got.sum() > 200 * 10**6


def test_perft5_equals_sum_of_children_perft4(engine, oracle):
    """All 200 roots of the split-pass test: perft(5)(root) == sum over the root's legal moves
    (oracle list + oracle next_state) of perft(4)(child), the children run through the OTHER
    leaf pass (GC_PERFT_SPLIT=0: depth-3 subtrees sorted by move count, k_perft_small_perm)."""
    import os

    b, m = _midgame_roots(200, 21, 0x5EED + 5)
    p5 = engine.perft(b, m, 5)
    kids_b, kids_m, owner = [], [], []
    for i in range(len(b)):
        for a in oracle.get_possible_moves(b[i], m[i], int(m[i, 0])):
            rc, nb, nm, _ = oracle.next_state(b[i], m[i], int(m[i, 0]), a)
            assert rc in (0, 1)
            kids_b.append(nb)
            kids_m.append(nm)
            owner.append(i)
    os.environ["GC_PERFT_SPLIT"] = "0"
    try:
        p4 = engine.perft(np.stack(kids_b), np.stack(kids_m), 4)
    finally:
        del os.environ["GC_PERFT_SPLIT"]
    sums = np.bincount(np.array(owner), weights=p4.astype(np.float64), minlength=len(b))
    assert (p5.astype(np.float64) == sums).all(), np.nonzero(p5.astype(np.float64) != sums)[0][:4]


def test_perft_chunked_levels_match(engine, oracle):
    """Levels too large to materialise are expanded one chunk of parents at a time (64-bit
    sizes; ADVICE r01: int32 level sums wrapped).  A 1 000-node level cap forces chunking at
    every expanded level; results == the unchunked run == the oracle."""
    import os

    b, m = _midgame_roots(48, 17, 0x5EED + 9)
    whole = engine.perft(b, m, 4)
    os.environ["GC_PERFT_LEVEL_CAP"] = "1000"
    try:
        chunked = engine.perft(b, m, 4)
    finally:
        del os.environ["GC_PERFT_LEVEL_CAP"]
    assert (whole == chunked).all()
    assert (whole == oracle.perft_batch(b, m, 4, threads=16)).all()


def test_perft6_startpos_vs_oracle(engine, oracle):
    """Depth 6 from the start position (four expanded levels, recursion through each): == the
    oracle (sum of perft(5) over the 20 children) == 124 483 101 (reference rules; FIDE is
    119 060 324 -- the difference is Q1, the double push over a blocker)."""
    from oracle import DEFAULT_BOARD, make_meta

    got = int(engine.perft(DEFAULT_BOARD[None], make_meta()[None], 6)[0])
    ref = int(oracle.perft_by_children(DEFAULT_BOARD[None], make_meta()[None], 6, threads=16)[0])
    assert got == ref == 124483101


# ------------------------------------------------------------------ env
def _replay_trace(env, oracle_env, steps):
    """Drive the batched env (1 board) with the recorded actions; compare to the golden."""
    from gym_chess_amd import codec as C

    for s in steps:
        if s["kind"] == "reset":
            env.reset()
            continue
        rw, dn, why = env.step([s["action"]])
        if s["kind"] == "error":
            assert why[0] == 5
            env.reset()
            continue
        assert rw[0] == s["reward"] and bool(dn[0]) == s["done"], s
        b, m = env.boards()
        assert C.board_to_text(b[0]) == s["board"]
        if "meta" in s:
            assert list(m[0, :7]) == s["meta"]
        assert m[0, 7] == s["move_count"]
        _, cnt = env.legal_moves()
        assert cnt[0] == s["n_moves"]


def test_env_traces_of_reference_env():
    """step() traces of the reference's ChessEnvV2 (opponent none; invalid actions; 3-fold;
    king capture / kingless play) replayed through gc_env_step."""
    from gym_chess_amd import codec as C
    from gym_chess_amd.env import BatchedChessEnv

    for t in load_golden("v2_env_traces.json.gz"):
        if t.get("opponent") == "random":
            continue
        ib = None if t["initial_board"] is None else C.text_to_board(t["initial_board"])
        env = BatchedChessEnv(1, device=0, seed=1, initial_board=ib)
        _replay_trace(env, None, t["steps"])


def test_env_batch_step_vs_oracle_env(oracle):
    """Many boards stepped in lockstep with external actions (valid and invalid)."""
    from gym_chess_amd.env import BatchedChessEnv

    n = 64
    env = BatchedChessEnv(n, device=0, seed=3)
    refs = [oracle.OracleEnv() for _ in range(n)]
    rng = np.random.RandomState(5)
    for ply in range(260):
        acts = np.zeros(n, dtype=np.int64)
        for i, r in enumerate(refs):
            mv = r.moves()
            if not mv or rng.rand() < 0.05:
                acts[i] = rng.randint(0, 4101)
            else:
                acts[i] = mv[rng.randint(len(mv))]
        rw, dn, why = env.step(acts)
        for i, r in enumerate(refs):
            rc, rr, rd, rq = r.step(int(acts[i]))
            if rc == 1:
                assert why[i] == 5
            else:
                assert rw[i] == rr and bool(dn[i]) == bool(rd), (ply, i)
        b, m = env.boards()
        for i, r in enumerate(refs):
            rb, rm = r.state()
            assert (b[i] == rb).all() and list(m[i]) == list(rm), (ply, i)
            if dn[i] or why[i] == 5:
                r.reset()
        resets = np.array([bool(dn[i]) or why[i] == 5 for i in range(n)], dtype=np.uint8)
        if resets.any():
            env.reset(resets)


@pytest.mark.parametrize("plies", [700])
def test_rollout_trajectories_vs_oracle(oracle, plies):
    """Fused rollout kernel: whole random self-play trajectories (incl. 3-fold, mate, move
    cap, no-move resets, king captures) bit-exact vs the oracle driver."""
    from gym_chess_amd.env import BatchedChessEnv

    n = 256
    env = BatchedChessEnv(n, device=0, seed=0xABCD)
    st, tr = env.rollout(plies, trace=True)
    ref_stats = np.zeros(8, dtype=np.uint64)
    for i in range(n):
        ref = oracle.rollout_trace(0xABCD, i, plies)
        for k in ("action", "reward", "done", "reason"):
            assert (tr[k][:, i] == ref[k]).all(), (i, k, np.nonzero(tr[k][:, i] != ref[k])[0][:3])
        ref_stats += ref["stats"]
    assert (st == ref_stats).all()
    b, m = env.boards()


def test_rollout_device_trace_vs_oracle(oracle):
    """gc_env_rollout_device (the bench's headline form: K steps in one launch, every ply's
    outputs in the device trace) vs the oracle driver: actions played, rewards, done, reasons
    of every ply and the final states.  200 boards: a partial last workgroup."""
    from gym_chess_amd.env import BatchedChessEnv

    n, plies, seed = 200, 500, 2024
    env = BatchedChessEnv(n, device=0, seed=seed)
    tb = env.trace_buffer(plies)
    env.rollout_device(plies, tb)
    env.synchronize()
    tr = tb.fetch()
    b, m = env.boards()
    for i in range(n):
        ref = oracle.rollout_trace(seed, i, plies)
        for k in ("action", "reward", "done", "reason"):
            assert (tr[k][:, i] == ref[k]).all(), (i, k, np.nonzero(tr[k][:, i] != ref[k])[0][:3])
        assert (b[i] == ref["final_board"]).all() and list(m[i]) == list(ref["final_meta"]), i


def test_rollout_device_past_one_launch(oracle):
    """More plies than one launch holds (ROLLOUT_MAX_PLIES = 16 383): the chunks continue one
    another exactly -- final states and next actions == the oracle's."""
    from concurrent.futures import ThreadPoolExecutor

    from gym_chess_amd.env import BatchedChessEnv

    n, plies, seed = 64, 16383 + 617, 55
    env = BatchedChessEnv(n, device=0, seed=seed)
    env.rollout_device(plies)
    b, m = env.boards()
    nxt = env.outputs()["next_action"]
    with ThreadPoolExecutor(8) as ex:
        refs = list(ex.map(lambda i: oracle.rollout_trace(seed, i, plies + 1), range(n)))
    for i, r in enumerate(refs):
        fin = oracle.rollout_trace(seed, i, plies)
        assert (b[i] == fin["final_board"]).all() and list(m[i]) == list(fin["final_meta"]), i
        assert nxt[i] == (0xFFFF if r["action"][plies] < 0 else r["action"][plies]), i


def test_step_random_matches_fused_rollout():
    """The one-ply step kernel (bench path) and the fused rollout kernel are the same driver."""
    from gym_chess_amd.env import BatchedChessEnv

    n, plies = 512, 400
    a = BatchedChessEnv(n, device=0, seed=99)
    bq = BatchedChessEnv(n, device=0, seed=99)
    a.step_random(plies)
    bq.rollout(plies)
    ba, ma = a.boards()
    bb, mb = bq.boards()
    assert (ba == bb).all() and (ma == mb).all()
    oa, ob = a.outputs(), bq.outputs()
    assert (oa["next_action"] == ob["next_action"]).all() and (oa["nsteps"] == ob["nsteps"]).all()


def test_step_random_per_ply_vs_oracle(oracle):
    """The bench kernel (k_env_step2, two waves per 64 boards) ply by ply: reward / done /
    reason of every ply and the next policy action, bit-exact vs the oracle driver.  200
    boards: the last workgroup is partial (dead lanes must reach the barriers)."""
    from gym_chess_amd.env import BatchedChessEnv

    n, plies, seed = 200, 320, 777
    env = BatchedChessEnv(n, device=0, seed=seed)
    refs = [oracle.rollout_trace(seed, i, plies + 1) for i in range(n)]
    ra = np.stack([r["action"] for r in refs], axis=1)
    rr = np.stack([r["reward"] for r in refs], axis=1)
    rd = np.stack([r["done"] for r in refs], axis=1)
    rq = np.stack([r["reason"] for r in refs], axis=1)
    for p in range(plies):
        env.step_random(1)
        o = env.outputs()
        nxt = np.where(ra[p + 1] < 0, 0xFFFF, ra[p + 1]).astype(np.uint16)
        assert (o["reward"] == rr[p]).all(), (p, np.nonzero(o["reward"] != rr[p])[0][:4])
        assert (o["done"] == rd[p]).all(), p
        assert (o["reason"] == rq[p]).all(), p  # incl. R_NO_MOVES (4) on a no-move reset ply
        assert (o["next_action"] == nxt).all(), (p, np.nonzero(o["next_action"] != nxt)[0][:4])


def _weird_initial_boards():
    """Initial boards the reference accepts but chess never has (several / no kings, pawns on
    the back rank, > 16 own pieces), for the bench kernel's reset and fallback paths."""
    from oracle import DEFAULT_BOARD

    boards, _ = random_positions(10, 4711)
    crowd = DEFAULT_BOARD.copy()  # 20 white pieces: the per-square fallback, no reset cache
    crowd[[33, 35, 37, 39]] = 2
    # 27 white queens round the edge and one inside, a black rook, no black king: 279 legal
    # moves for white, past the byte-sum pick (the set-wise pick's rolled scan)
    queens = np.zeros(64, dtype=np.int8)
    queens[[1, 2, 3, 4, 5, 6, 7, 8, 15, 16, 23, 24, 31, 32, 36, 39, 40, 47, 48, 55, 56, 57, 58, 59, 60, 61, 62]] = 2
    queens[63], queens[0] = 1, -3
    return list(boards) + [crowd, queens]


@pytest.mark.parametrize("k", range(12))
def test_step_random_weird_initial_boards_vs_oracle(oracle, k):
    """k_env_step2 ply by ply from (and resetting to) a weird initial board: outputs, next
    action and final states vs the oracle driver with the same initial board.  70 boards:
    a partial second workgroup."""
    from gym_chess_amd.env import BatchedChessEnv

    ib = _weird_initial_boards()[k]
    n, plies, seed = 70, 90, 1000 + k
    env = BatchedChessEnv(n, device=0, seed=seed, initial_board=ib)
    refs = [oracle.rollout_trace(seed, i, plies + 1, init=ib) for i in range(n)]
    ra = np.stack([r["action"] for r in refs], axis=1)
    for p in range(plies):
        env.step_random(1)
        o = env.outputs()
        nxt = np.where(ra[p + 1] < 0, 0xFFFF, ra[p + 1]).astype(np.uint16)
        for key, name in (("reward", "reward"), ("done", "done"), ("reason", "reason")):
            want = np.stack([r[name][p] for r in refs])
            assert (o[key] == want).all(), (k, p, key, np.nonzero(o[key] != want)[0][:4])
        assert (o["next_action"] == nxt).all(), (k, p, np.nonzero(o["next_action"] != nxt)[0][:4])
    b, m = env.boards()
    fin = [oracle.rollout_trace(seed, i, plies, init=ib) for i in range(n)]
    for i in range(n):
        assert (b[i] == fin[i]["final_board"]).all() and list(m[i]) == list(fin[i]["final_meta"]), (k, i)


@pytest.mark.parametrize("k", range(12))
def test_fused_rollouts_weird_initial_boards_vs_oracle(oracle, k):
    """The fused rollouts (rollout(trace=True) and rollout_device with a device trace) from and
    resetting to every weird initial board: each ply's action / reward / done / reason, the next
    action and the final states vs the oracle driver (chess_v2.py:183-217 resets to
    initial_board; test_benchmark.py:17-31 drives it).  The crowd board (> 16 own pieces) and the
    279-queens board have no reset pick table, so they must not run on the quads (whose reset
    pick is the table's) -- rollout_waves says which kernel runs."""
    from gym_chess_amd.env import BatchedChessEnv

    ib = _weird_initial_boards()[k]
    n, plies, seed = 70, 300, 2000 + k
    refs = [oracle.rollout_trace(seed, i, plies + 1, init=ib) for i in range(n)]
    fin = [oracle.rollout_trace(seed, i, plies, init=ib) for i in range(n)]
    want = {name: np.stack([r[name][:plies] for r in refs], axis=1) for name in ("action", "reward", "done", "reason")}
    nxt = np.array([0xFFFF if r["action"][plies] < 0 else r["action"][plies] for r in refs], dtype=np.uint16)
    for form in ("rollout", "device"):
        env = BatchedChessEnv(n, device=0, seed=seed, initial_board=ib)
        if k >= 10:  # the crowd and queens boards: no table, the paired kernel
            assert env.rollout_waves() == 2, (k, env.rollout_waves())
        if form == "rollout":
            _, tr = env.rollout(plies, trace=True)
        else:
            buf = env.trace_buffer(plies)
            env.rollout_device(plies, trace=buf)
            tr = buf.fetch()
            buf.close()
        for name in ("action", "reward", "done", "reason"):
            got = tr[name]
            bad = np.argwhere(got != want[name])
            assert bad.size == 0, (k, form, name, bad[:4].tolist())
        assert (env.outputs()["next_action"] == nxt).all(), (k, form)
        b, m = env.boards()
        for i in range(n):
            assert (b[i] == fin[i]["final_board"]).all() and list(m[i]) == list(fin[i]["final_meta"]), (k, form, i)
        env.close()


def test_fused_rollout_stats_and_states_vs_oracle(oracle):
    """The paired fused-rollout kernel (k_env_rollout2, no trace): per-board final states and
    the aggregate episode stats of 200 boards x 500 plies == the oracle driver's."""
    from gym_chess_amd.env import BatchedChessEnv

    n, plies, seed = 200, 500, 31337
    env = BatchedChessEnv(n, device=0, seed=seed)
    st, _ = env.rollout(plies)
    b, m = env.boards()
    ref = np.zeros(8, dtype=np.uint64)
    for i in range(n):
        r = oracle.rollout_trace(seed, i, plies)
        ref += r["stats"]
        assert (b[i] == r["final_board"]).all() and list(m[i]) == list(r["final_meta"]), i
    assert (st == ref).all(), (st, ref)


def test_step_random_vs_oracle_final_state(oracle):
    from gym_chess_amd.env import BatchedChessEnv

    n, plies = 128, 333
    env = BatchedChessEnv(n, device=0, seed=4242)
    env.step_random(plies)
    b, m = env.boards()
    for i in range(n):
        ref = oracle.rollout_trace(4242, i, plies)
        assert (b[i] == ref["final_board"]).all() and list(m[i]) == list(ref["final_meta"]), i


def test_legal_mask_matches_list():
    from gym_chess_amd.env import BatchedChessEnv

    env = BatchedChessEnv(256, device=0, seed=8)
    env.step_random(57)
    mask = env.legal_mask()
    acts = env.possible_actions()
    for i in range(256):
        assert sorted(np.nonzero(mask[i])[0].tolist()) == sorted(acts[i])


def test_chess_engine_compat_dict_api(oracle):
    """The drop-in ChessEngine: same dict/str protocol as lib.rs."""
    from gym_chess_amd import codec as C
    from gym_chess_amd.engine import ChessEngine

    eng = ChessEngine()
    state = dict(board=C.DEFAULT_BOARD, current_player="WHITE", white_king_castle_is_possible=True,
                 white_queen_castle_is_possible=True, black_king_castle_is_possible=True,
                 black_queen_castle_is_possible=True)
    st = eng.update_state(state)
    assert st["white_king_is_checked"] is False and st["board"] == C.DEFAULT_BOARD
    moves = eng.get_possible_moves(st, "WHITE")
    assert moves[:4] == ["a2a3", "a2a4", "b2b3", "b2b4"] and len(moves) == 20
    ns, rw = eng.next_state(st, "WHITE", "e2e4")
    assert ns["current_player"] == "BLACK" and rw == 0 and ns["board"][4][4] == 6
    with pytest.raises(SystemError):
        eng.get_possible_moves(st, "RED")
    with pytest.raises(KeyError):
        eng.get_possible_moves({"board": C.DEFAULT_BOARD}, "WHITE")
    assert eng.get_castle_moves(st, "WHITE") == []


@pytest.mark.parametrize("n", [70, 200, 1000])
def test_step_random_board_range_streams_agree(n):
    """gc_env_step_random over 1, 2 and 3 board-range streams (ranges are whole workgroups of
    PAIRS_WG blocks; the last one partial): identical states and outputs."""
    from gym_chess_amd.env import BatchedChessEnv

    res = []
    for k in (1, 2, 3):
        env = BatchedChessEnv(n, device=0, seed=4040)
        env.set_streams(k)
        env.step_random(333)
        b, m = env.boards()
        res.append((b, m, env.outputs()))
        env.close()
    for b, m, o in res[1:]:
        assert (b == res[0][0]).all() and (m == res[0][1]).all()
        for key in o:
            assert (o[key] == res[0][2][key]).all(), key
