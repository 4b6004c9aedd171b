"""CPU differential tests of the product's bitboard core (the exact device code of
gc_core.h / gc_env.h, host-compiled) against the oracle.  The GPU tests repeat the
important ones through the real kernels."""
import os
import sys

import numpy as np
import pytest

from conftest import load_golden, random_positions

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "core_host"))
import corehost as H  # noqa: E402


def naive_between(a, b):
    ra, ca = divmod(a, 8)
    rb, cb = divmod(b, 8)
    dr, dc = rb - ra, cb - ca
    if a == b or not (dr == 0 or dc == 0 or abs(dr) == abs(dc)):
        return 0
    sr, sc = (dr > 0) - (dr < 0), (dc > 0) - (dc < 0)
    m, r, c = 0, ra + sr, ca + sc
    while (r, c) != (rb, cb):
        m |= 1 << (r * 8 + c)
        r += sr
        c += sc
    return m


def naive_slide(sq, occ, dirs):
    m = 0
    r0, c0 = divmod(sq, 8)
    for dr, dc in dirs:
        r, c = r0 + dr, c0 + dc
        while 0 <= r < 8 and 0 <= c < 8:
            m |= 1 << (r * 8 + c)
            if occ >> (r * 8 + c) & 1:
                break
            r += dr
            c += dc
    return m


def test_between_exhaustive():
    L = H.lib()
    for a in range(64):
        for b in range(64):
            assert L.host_between(a, b) == naive_between(a, b), (a, b)


def test_slider_attacks_random_occupancy():
    L = H.lib()
    rng = np.random.RandomState(0)
    for _ in range(5000):
        occ = int(rng.randint(0, 2**63, dtype=np.int64)) & int(rng.randint(0, 2**63, dtype=np.int64))
        sq = int(rng.randint(64))
        assert L.host_rook_att(sq, occ) == naive_slide(sq, occ, [(1, 0), (-1, 0), (0, 1), (0, -1)])
        assert L.host_bishop_att(sq, occ) == naive_slide(sq, occ, [(1, 1), (-1, 1), (1, -1), (-1, -1)])


def test_v1_games(oracle):
    from gym_chess_amd import codec as C

    for g in load_golden("v1_games.json.gz"):
        for p in g["plies"]:
            b = C.text_to_board(p["board"])
            m = oracle.make_meta(p["white"], *p["rights"])
            assert H.get_list(b, m, p["white"]) == p["moves"]
            assert H.get_list_emit(b, m, p["white"]) == p["moves"]


def test_perft_startpos(oracle):
    b, m = oracle.DEFAULT_BOARD, oracle.make_meta()
    assert [H.perft(b, m, d) for d in range(1, 5)] == [20, 400, 8982, 200915]


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_fuzz_positions(oracle, seed):
    boards, metas = random_positions(300, seed)
    rng = np.random.RandomState(seed)
    for i in range(len(boards)):
        b, m = boards[i], metas[i]
        for white in (0, 1):
            ref = oracle.get_possible_moves(b, m, white)
            assert H.get_list(b, m, white) == ref, (i, white)
            assert H.get_list_emit(b, m, white) == ref, (i, white)  # for_targets_ordered (list_one / list_par)
            assert H.count(b, m, white) == len(ref)
            assert H.count2(b, m, white) == len(ref)
            srt = sorted(ref)
            for k in range(len(ref)):
                assert H.select(b, m, white, k) == ref[k]
                assert H.select2(b, m, white, k) == ref[k]
                assert H.select_action(b, m, white, k) == srt[k]  # the policy's action-id order
            legal = set(ref)
            for a in list(legal)[:5] + [int(x) for x in rng.randint(0, 4101, size=5)]:
                assert H.action_legal(b, m, white, a) == (a in legal)
            assert H.get_list(b, m, white, attack=True) == oracle.get_possible_moves(b, m, white, True)
            assert H.get_list_emit(b, m, white, attack=True) == oracle.get_possible_moves(b, m, white, True)
        rb, rm = oracle.update_state(b, m)
        hb, hm = H.update_state(b, m)
        assert list(hm[:7]) == list(rm[:7])
        occupied = np.nonzero(b)[0]
        for _ in range(4):
            a = int(rng.choice(occupied)) * 64 + int(rng.randint(64)) if rng.rand() < 0.8 else 4096 + int(rng.randint(4))
            pw = int(rng.randint(2))
            r1 = oracle.next_state(b, m, pw, a)
            r2 = H.next_state(b, m, pw, a)
            assert r1[0] == r2[0]
            if r1[0] in (0, 1):
                assert (r1[1] == r2[1]).all() and list(r1[2][:7]) == list(r2[2][:7]) and r1[3] == r2[3]


def test_fuzz_perft(oracle):
    boards, metas = random_positions(40, 77)
    for i in range(len(boards)):
        for d in (1, 2, 3):
            ref = oracle.perft(boards[i], metas[i], d)
            assert H.perft(boards[i], metas[i], d) == ref, (i, d)
            assert H.perft_small(boards[i], metas[i], d) == ref, (i, d)


def test_perft_small_startpos(oracle):
    b, m = oracle.DEFAULT_BOARD, oracle.make_meta()
    assert [H.perft_small(b, m, d) for d in range(0, 5)] == [1, 20, 400, 8982, 200915]


def test_rollout_trajectories(oracle):
    for bid in range(120):
        ref = oracle.rollout_trace(0x1234, bid, 700)
        got = H.rollout_trace(0x1234, bid, 700, oracle.DEFAULT_BOARD)
        for k in ("action", "reward", "done", "reason", "final_board", "final_meta", "stats"):
            assert (got[k] == ref[k]).all(), (bid, k)


def test_rollout_from_custom_initial_board(oracle):
    """Kingless / odd initial boards through the same driver."""
    boards, _ = random_positions(12, 5)
    for i, b in enumerate(boards):
        ref = oracle.rollout_trace(9, i, 400, init=b)
        got = H.rollout_trace(9, i, 400, b)
        for k in ("action", "reward", "done", "reason", "final_board", "final_meta", "stats"):
            assert (got[k] == ref[k]).all(), (i, k)


def test_env_traces(oracle):
    from gym_chess_amd import codec as C

    for t in load_golden("v2_env_traces.json.gz"):
        if t.get("opponent") == "random":
            continue
        init = oracle.DEFAULT_BOARD if t["initial_board"] is None else C.text_to_board(t["initial_board"])
        e = H.HostEnv(init)
        for s in t["steps"]:
            if s["kind"] == "reset":
                e.reset()
                continue
            rc, rw, dn, why = e.step(s["action"])
            if s["kind"] == "error":
                assert rc == 1
                e.reset()
                continue
            assert rw == s["reward"] and bool(dn) == s["done"], s
            b, m = e.state()
            assert C.board_to_text(b) == s["board"] and m[7] == s["move_count"]
            assert len(e.moves()) == s["n_moves"]


def test_mover_check_shortcut_every_legal_move():
    """The step's mover check flag (mover_checked: false for non-king moves, x-ray along the
    line through the king's squares or a captured enemy king's pawn-attacked square for king
    moves, the full probe for castles / several kings) == the full attack probe, on every
    legal move of weird random positions (several / no kings, castling geometry)."""
    hits = {"king_move_checked": 0, "castle_or_multi": 0, "moves": 0}
    for seed in (71, 72, 73):
        boards, metas = random_positions(1500, seed)
        for b, m in zip(boards, metas):
            white = int(m[0])
            for a in H.get_list(b, m, white):
                short, full = H.mover_checked(b, m, a)
                assert short == full, (seed, b.tolist(), m.tolist(), a)
                hits["moves"] += 1
                hits["king_move_checked"] += a < 4096 and full
                hits["castle_or_multi"] += a >= 4096
    # the interesting cases occur (Q6 retreats along a checking ray, castles)
    assert hits["king_move_checked"] > 50 and hits["castle_or_multi"] > 50, hits


@pytest.mark.parametrize("seed", [11, 12])
def test_count_moves_agrees(seed):
    """count_moves (perft leaves: set-wise sliders / knights) == gen_moves' total ==
    count_legal on fuzz positions (several / no kings, pins, checks), both sides to move."""
    from conftest import random_positions

    boards, metas = random_positions(3000, seed)
    L = H.lib()
    seen = 0
    for i in range(len(boards)):
        for white in (0, 1):
            c = L.host_count_moves_agree(boards[i].ctypes.data, metas[i].ctypes.data, white)
            assert c >= 0, (i, white, -1 - c)
            seen += c
    assert seen > 0


@pytest.mark.parametrize("seed", [16, 17])
def test_setwise_generation_agrees(seed):
    """Set-wise generation (sw_gen: pawn / knight / king / slider-direction target sets, the
    self-play policy's move-set order): its count == count_legal, and sw_select over every
    rank yields each legal action exactly once, on fuzz positions (several / no kings, pins,
    checks, > 16 pieces), both sides to move."""
    from conftest import random_positions

    boards, metas = random_positions(3000, seed)
    L = H.lib()
    seen = 0
    for i in range(len(boards)):
        for white in (0, 1):
            c = L.host_sw_agree(boards[i].ctypes.data, metas[i].ctypes.data, white)
            assert c >= 0, (i, white, c)
            seen += c
    assert seen > 0


@pytest.mark.parametrize("seed", [14, 15])
def test_swar_pick_agrees(seed):
    """select_action_swar (byte-wise prefix sums of the count planes) == select_action (the
    bisection) for every rank on fuzz positions, both sides to move."""
    from conftest import random_positions

    boards, metas = random_positions(3000, seed)
    L = H.lib()
    ranks = 0
    for i in range(len(boards)):
        for white in (0, 1):
            c = L.host_pick_agree(boards[i].ctypes.data, metas[i].ctypes.data, white)
            assert c >= 0, (i, white, -1 - c)
            ranks += c
    assert ranks > 10000


@pytest.mark.parametrize("seed,weird", [(13, True), (14, False)])
def test_quick_legal_agrees(seed, weird):
    """quick_legal (the paired API step's validation: no enemy map, a king target's attack
    test alone) and its two halves quick_pseudo && quick_safe (the quad API step's, on two
    waves) == action_legal over gen_init for all 4 101 action ids (and -1, 4101, larger ids)
    on fuzz positions, both sides to move."""
    from conftest import random_positions

    boards, metas = random_positions(600, seed, weird=weird)
    L = H.lib()
    legal = 0
    for i in range(len(boards)):
        for white in (0, 1):
            c = L.host_quick_legal_agree(boards[i].ctypes.data, metas[i].ctypes.data, white)
            assert c >= 0, (i, white, -1 - c)
            legal += c
    assert legal > 1000


@pytest.mark.parametrize("seed", [51, 52, 53])
def test_pin_forms_agree(seed):
    """gen_pins_aligned (the aligned-slider loop the kernels run) == gen_pins_part (the
    four-line x-ray form) on fuzz positions, both sides to move: in check, check mask,
    pinned, pin rays."""
    from conftest import random_positions

    boards, metas = random_positions(3000, seed)
    L = H.lib()
    for i in range(len(boards)):
        for white in (0, 1):
            assert L.host_pins_agree(boards[i].ctypes.data, metas[i].ctypes.data, white) == 1, (i, white)


# Two pins on one line through the king -- a rook behind it pinning one pawn, a queen in front
# pinning another -- and the rear pawn's Q1 double push jumps the king onto the FRONT pin's
# segment (pinrays is the union of the segments).  The reference's legality filter rejects the
# move (the rook then checks the king); found at ply 4 591 of board 65 486, seed 1000, by the
# 20 000-ply soak (tools/soak.py).
TWO_PINS = (
    "..b.kb.."
    "..p..qp."
    "n.np...r"
    ".pP.pP.p"
    "Pp..N..."
    "..B..K.."
    ".....P.R"
    ".....rN."
)


def _two_pins_position(mirror=False):
    from gym_chess_amd import codec as C

    b = C.text_to_board(TWO_PINS)
    m = np.zeros(8, dtype=np.uint8)
    m[0], m[3], m[4] = 1, 1, 1
    if mirror:  # colours swapped and the board flipped: black's pawn jumps its king
        b = -b.reshape(8, 8)[::-1].reshape(64)
        m[0], m[1], m[2], m[3], m[4] = 0, 1, 1, 0, 0
    return b.astype(np.int8), m


@pytest.mark.parametrize("mirror", [False, True])
def test_pinned_pawn_double_push_never_crosses_its_king(oracle, mirror):
    b, m = _two_pins_position(mirror)
    w = int(m[0])
    ref = oracle.get_possible_moves(b, m, w)
    assert H.get_list(b, m, w) == ref
    assert H.count(b, m, w) == len(ref) == H.count2(b, m, w)
    jump = (53 * 64 + 37) if not mirror else (13 * 64 + 29)  # f2-f4 / f7-f5 over the king
    assert jump not in ref and not H.action_legal(b, m, w, jump)
    for d in (1, 2, 3):
        assert H.perft(b, m, d) == oracle.perft(b, m, d)


def test_soak_board_65486_trajectory(oracle):
    from gym_chess_amd import codec as C

    init = np.array(C.DEFAULT_BOARD, np.int8).reshape(64)
    o = oracle.rollout_trace(1000, 65486, 4600)
    h = H.rollout_trace(1000, 65486, 4600, init)
    assert (o["action"] == h["action"]).all() and (o["final_board"] == h["final_board"]).all()
