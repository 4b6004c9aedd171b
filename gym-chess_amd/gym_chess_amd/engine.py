"""Engine API on the GPU.

* `Engine`      -- batched numpy API over gc_engine_* (many positions per launch).
* `ChessEngine` -- drop-in for the reference's PyO3 class `gym_chess.ChessEngine`
                   (/root/reference/src/lib.rs:1412-1512): same four methods, same dict /
                   "e2e4"-string conventions, same error behaviour, one GPU launch per call.

Reference call sites this replaces: chess_v2.py:146 (construction), 204 (update_state),
419 (next_state), 579 (get_possible_moves), 590 (get_castle_moves).
"""
import ctypes
import threading

import numpy as np

from . import _lib
from . import codec as C

MAX_LIST = 320  # > the largest legal move list of any position reachable by the engine


class Engine:
    """Batched stateless engine on one device.  States are (boards int8[n,64], meta uint8[n,8]).

    rules="fide" (not the reference's rules): en passant, promotion,
    per-side castling, no king captures; meta[7] is then the en-passant file + 1 (0 = none),
    lists are in ascending action id with castles last, perft counts the four promotions."""

    def __init__(self, device=0, rules="reference"):
        self._L = _lib.load()
        rid = _lib.rules_id(rules)
        h = ctypes.c_void_p()
        _lib.check(self._L.gc_engine_create(int(device), ctypes.byref(h)))
        self._h = h
        self.device = device
        self.rules = rules
        _lib.check(self._L.gc_engine_set_rules(self._h, rid))

    def close(self):
        if getattr(self, "_h", None):
            self._L.gc_engine_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @staticmethod
    def _prep(boards, meta):
        b = np.ascontiguousarray(boards, dtype=np.int8).reshape(-1, 64)
        m = np.ascontiguousarray(meta, dtype=np.uint8).reshape(-1, 8)
        if b.shape[0] != m.shape[0]:
            raise ValueError("boards and meta must have the same batch size")
        return b, m

    @staticmethod
    def _players(player_white, n):
        p = np.ascontiguousarray(np.broadcast_to(np.asarray(player_white, dtype=np.uint8), (n,)))
        return p

    def possible_moves(self, boards, meta, player_white, attack=False, cap=MAX_LIST):
        """-> (moves uint16[n, cap], counts int32[n]) in reference order."""
        b, m = self._prep(boards, meta)
        n = b.shape[0]
        p = self._players(player_white, n)
        out = np.zeros((n, cap), dtype=np.uint16)
        cnt = np.zeros(n, dtype=np.int32)
        _lib.check(self._L.gc_engine_get_possible_moves(self._h, n, _lib.ptr(b), _lib.ptr(m), _lib.ptr(p),
                                                        int(bool(attack)), _lib.ptr(out), int(cap), _lib.ptr(cnt)))
        return out, cnt

    def castle_moves(self, boards, meta, player_white):
        b, m = self._prep(boards, meta)
        n = b.shape[0]
        p = self._players(player_white, n)
        out = np.zeros((n, 2), dtype=np.uint16)
        cnt = np.zeros(n, dtype=np.int32)
        _lib.check(self._L.gc_engine_get_castle_moves(self._h, n, _lib.ptr(b), _lib.ptr(m), _lib.ptr(p),
                                                      _lib.ptr(out), _lib.ptr(cnt)))
        return out, cnt

    def next_state(self, boards, meta, player_white, actions):
        """-> (boards, meta, rewards int32[n], status int32[n])"""
        b, m = self._prep(boards, meta)
        n = b.shape[0]
        p = self._players(player_white, n)
        a = np.ascontiguousarray(np.broadcast_to(np.asarray(actions, dtype=np.uint16), (n,)))
        ob = np.zeros((n, 64), dtype=np.int8)
        om = np.zeros((n, 8), dtype=np.uint8)
        rw = np.zeros(n, dtype=np.int32)
        st = np.zeros(n, dtype=np.int32)
        _lib.check(self._L.gc_engine_next_state(self._h, n, _lib.ptr(b), _lib.ptr(m), _lib.ptr(p), _lib.ptr(a),
                                                _lib.ptr(ob), _lib.ptr(om), _lib.ptr(rw), _lib.ptr(st)))
        return ob, om, rw, st

    def update_state(self, boards, meta):
        b, m = self._prep(boards, meta)
        n = b.shape[0]
        ob = np.zeros((n, 64), dtype=np.int8)
        om = np.zeros((n, 8), dtype=np.uint8)
        _lib.check(self._L.gc_engine_update_state(self._h, n, _lib.ptr(b), _lib.ptr(m), _lib.ptr(ob), _lib.ptr(om)))
        return ob, om

    def perft(self, boards, meta, depth):
        b, m = self._prep(boards, meta)
        n = b.shape[0]
        out = np.zeros(n, dtype=np.uint64)
        _lib.check(self._L.gc_engine_perft(self._h, n, _lib.ptr(b), _lib.ptr(m), int(depth), _lib.ptr(out)))
        return out


def perft_path_counts():
    """Diagnostics: {pass: runs in this process} of the perft leaf passes (gc_perft_path_counts)."""
    out = np.zeros(4, dtype=np.uint64)
    _lib.check(_lib.load().gc_perft_path_counts(_lib.ptr(out)))
    return dict(zip(("split", "sorted", "small", "fide"), (int(x) for x in out)))


class ChessEngine:
    """Drop-in replacement for the reference's `gym_chess.ChessEngine` (lib.rs:1412-1512).

    Errors mirror the reference: a missing state key raises (the Rust side unwrap()s);
    a bad colour or a both-kings-checked result raises SystemError (PyO3 returns Ok with a
    Python exception set, lib.rs:434-437, 1442-1446); an empty from-square raises
    (Rust panic, lib.rs:693-695).
    """

    def __init__(self, device=0):
        self._e = Engine(device)
        # one position per call: the outputs' buffers made once (their pointers too); the
        # result is converted to Python objects before the call returns
        self._moves = np.zeros(MAX_LIST, dtype=np.uint16)
        self._cnt = np.zeros(1, dtype=np.int32)
        self._white = (np.ones(1, dtype=np.uint8), np.zeros(1, dtype=np.uint8))
        self._p_moves, self._p_cnt = _lib.ptr(self._moves), _lib.ptr(self._cnt)
        self._p_white = (_lib.ptr(self._white[0]), _lib.ptr(self._white[1]))
        self._act = np.zeros(1, dtype=np.uint16)
        self._ob = np.zeros(64, dtype=np.int8)
        self._om = np.zeros(8, dtype=np.uint8)
        self._rw = np.zeros(1, dtype=np.int32)
        self._st = np.zeros(1, dtype=np.int32)
        self._p_act, self._p_ob, self._p_om = _lib.ptr(self._act), _lib.ptr(self._ob), _lib.ptr(self._om)
        self._p_rw, self._p_st = _lib.ptr(self._rw), _lib.ptr(self._st)
        # the buffers above are shared by every call on this instance, and ctypes releases the
        # GIL inside the C call: one call at a time, from the inputs' staging through the
        # conversion of the outputs to Python objects
        self._lock = threading.Lock()

    def next_state(self, state, player, move):
        b, m = C.dict_to_arrays(state)
        white = self._player(player)
        act = C.str_to_action(move)
        e = self._e
        with self._lock:
            self._act[0] = act
            _lib.check(e._L.gc_engine_next_state(e._h, 1, _lib.ptr(b), _lib.ptr(m), self._p_white[0 if white else 1],
                                                 self._p_act, self._p_ob, self._p_om, self._p_rw, self._p_st))
            st = int(self._st[0])
            if st == 0:
                return C.arrays_to_dict(self._ob, self._om), int(self._rw[0])
        if st == -1:
            raise RuntimeError("Bad move - piece is empty !")
        if st == 1:
            raise SystemError("Both Kings are in check: this position is impossible")
        raise ValueError(f"bad move {move!r}")

    def get_possible_moves(self, state, player, attack=False):
        b, m = C.dict_to_arrays(state)
        white = self._player(player)
        e = self._e
        with self._lock:
            _lib.check(e._L.gc_engine_get_possible_moves(e._h, 1, _lib.ptr(b), _lib.ptr(m),
                                                         self._p_white[0 if white else 1], 1 if attack else 0,
                                                         self._p_moves, MAX_LIST, self._p_cnt))
            n = int(self._cnt[0])
            if n <= MAX_LIST:
                return C.actions_to_strs(self._moves[:n])
        out, cnt = e.possible_moves(b, m, white, attack, cap=n)  # fresh output arrays
        return C.actions_to_strs(out[0, :n])

    def get_castle_moves(self, state, player):
        b, m = C.dict_to_arrays(state)
        white = self._player(player)
        e = self._e
        with self._lock:
            _lib.check(e._L.gc_engine_get_castle_moves(e._h, 1, _lib.ptr(b), _lib.ptr(m),
                                                       self._p_white[0 if white else 1], self._p_moves, self._p_cnt))
            return C.actions_to_strs(self._moves[: int(self._cnt[0])])

    def update_state(self, state):
        b, m = C.dict_to_arrays(state)
        e = self._e
        with self._lock:
            _lib.check(e._L.gc_engine_update_state(e._h, 1, _lib.ptr(b), _lib.ptr(m), self._p_ob, self._p_om))
            return C.arrays_to_dict(self._ob, self._om)

    @staticmethod
    def _player(player):
        try:
            return C.player_to_white(player)
        except ValueError as ex:  # lib.rs:433-437
            raise SystemError(str(ex)) from None


def perft_leaf_stats():
    """Diagnostics: the split pass's leaf kernel in this process -> (launches, subtrees, kernel ms)."""
    la, st, ms = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_double()
    _lib.check(_lib.load().gc_perft_leaf_stats(ctypes.byref(la), ctypes.byref(st), ctypes.byref(ms)))
    return int(la.value), int(st.value), float(ms.value)


def perft_dedup_stats():
    """Diagnostics: the split pass's depth-2 roots in this process -> (records made, subtrees
    counted); counted < records when the transposition pass merged equal positions."""
    r, c = ctypes.c_uint64(), ctypes.c_uint64()
    _lib.check(_lib.load().gc_perft_dedup_stats(ctypes.byref(r), ctypes.byref(c)))
    return int(r.value), int(c.value)
