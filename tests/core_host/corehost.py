"""TEST INFRASTRUCTURE ONLY -- ctypes view of the host build of the product's bitboard core
(gym-chess_amd/csrc/gc_core.h + gc_env.h compiled by g++), for CPU differential tests."""
import ctypes
import hashlib
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "libcorehost.so")
_STAMP = _SO + ".srchash"
_CSRC = os.path.join(_HERE, "..", "..", "gym-chess_amd", "csrc")
FLAGS = ["-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-Wno-unknown-pragmas"]
_L = None
P = ctypes.c_void_p


def source_hash():
    """sha256 prefix of core_host.cpp, the product's device headers it compiles and the flags
    (content, not mtimes: a library built from other sources is never reused)"""
    h = hashlib.sha256(" ".join(FLAGS).encode())
    srcs = [os.path.join(_HERE, "core_host.cpp")] + sorted(
        os.path.join(_CSRC, f) for f in os.listdir(_CSRC) if f.endswith(".h"))
    for path in srcs:
        h.update(os.path.basename(path).encode() + b"\0")
        with open(path, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def ensure_built():
    """(re)build libcorehost.so unless its stamp holds the current source hash"""
    want = source_hash()
    if os.path.exists(_SO) and os.path.exists(_STAMP) and open(_STAMP).read().strip() == want:
        return
    os.makedirs(os.path.dirname(_SO), exist_ok=True)
    tmp = f"{_SO}.{os.getpid()}.tmp"  # build aside, then rename: parallel test workers never load a partial file
    subprocess.run(["g++"] + FLAGS + ["-o", tmp, os.path.join(_HERE, "core_host.cpp")], check=True)
    os.replace(tmp, _SO)
    with open(f"{_STAMP}.{os.getpid()}.tmp", "w") as f:
        f.write(want)
    os.replace(f"{_STAMP}.{os.getpid()}.tmp", _STAMP)


def lib():
    global _L
    if _L is None:
        ensure_built()
        L = ctypes.CDLL(_SO)
        L.host_between.restype = ctypes.c_uint64
        L.host_pins_agree.argtypes = [P, P, ctypes.c_int]
        L.host_count_moves_agree.argtypes = [P, P, ctypes.c_int]
        L.host_quick_legal_agree.argtypes = [P, P, ctypes.c_int]
        L.host_pick_agree.argtypes = [P, P, ctypes.c_int]
        L.host_sw_agree.argtypes = [P, P, ctypes.c_int]
        L.host_rook_att.restype = ctypes.c_uint64
        L.host_rook_att.argtypes = [ctypes.c_int, ctypes.c_uint64]
        L.host_bishop_att.restype = ctypes.c_uint64
        L.host_bishop_att.argtypes = [ctypes.c_int, ctypes.c_uint64]
        L.host_side_attacks.restype = ctypes.c_uint64
        L.host_side_attacks.argtypes = [P, ctypes.c_int]
        L.host_perft.restype = ctypes.c_uint64
        L.host_perft.argtypes = [P, P, ctypes.c_int]
        L.host_perft_small.restype = ctypes.c_uint64
        L.host_perft_small.argtypes = [P, P, ctypes.c_int]
        L.host_list.argtypes = [P, P, ctypes.c_int, ctypes.c_int, P, ctypes.c_int]
        L.host_list_emit.argtypes = [P, P, ctypes.c_int, ctypes.c_int, P, ctypes.c_int]
        L.host_count.argtypes = [P, P, ctypes.c_int]
        L.host_count2.argtypes = [P, P, ctypes.c_int]
        L.host_select2.argtypes = [P, P, ctypes.c_int, ctypes.c_int]
        L.host_select_action.argtypes = [P, P, ctypes.c_int, ctypes.c_int]
        L.host_select.argtypes = [P, P, ctypes.c_int, ctypes.c_int]
        L.host_action_legal.argtypes = [P, P, ctypes.c_int, ctypes.c_int]
        L.host_next_state.argtypes = [P, P, ctypes.c_int, ctypes.c_int, P, P, P]
        L.host_mover_checked.argtypes = [P, P, ctypes.c_int]
        L.host_update_state.argtypes = [P, P, P, P]
        L.host_rollout_trace.argtypes = [P, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, P, P, P, P, P, P, P]
        L.host_env_new.restype = P
        L.host_env_new.argtypes = [P]
        L.host_env_new2.restype = P
        L.host_env_new2.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint32]
        L.host_env_pick.argtypes = [P]
        L.host_env_pick.restype = ctypes.c_int
        L.host_env_draw.argtypes = [P]
        L.host_env_draw.restype = ctypes.c_uint32
        L.host_rollout_trace2.argtypes = [P, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_int, P, P, P, P, P, P, P]
        L.host_env_free.argtypes = [P]
        L.host_env_reset.argtypes = [P]
        L.host_env_step.argtypes = [P, ctypes.c_int, P, P, P]
        L.host_env_state.argtypes = [P, P, P]
        L.host_env_moves.argtypes = [P, P, ctypes.c_int]
        L.host_fide_perft.restype = ctypes.c_uint64
        L.host_fide_perft.argtypes = [P, P, ctypes.c_int]
        L.host_fide_gen_check.argtypes = [P, P, ctypes.c_int, P, P, P]
        L.host_fide_list.argtypes = [P, P, P, ctypes.c_int]
        L.host_fide_rollout.argtypes = [P, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, P, P, P, P]
        _L = L
    return _L


def _p(a):
    return a.ctypes.data_as(P)


def _bm(b, m):
    return np.ascontiguousarray(b, dtype=np.int8).reshape(64), np.ascontiguousarray(m, dtype=np.uint8).reshape(8)


def get_list(board, meta, white, attack=False):
    b, m = _bm(board, meta)
    out = np.zeros(1024, dtype=np.uint16)
    n = lib().host_list(_p(b), _p(m), int(white), int(bool(attack)), _p(out), 1024)
    return [int(x) for x in out[:n]]


def get_list_emit(board, meta, white, attack=False):
    """get_list through for_targets_ordered (the device's one-pass emit)"""
    b, m = _bm(board, meta)
    out = np.zeros(1024, dtype=np.uint16)
    n = lib().host_list_emit(_p(b), _p(m), int(white), int(bool(attack)), _p(out), 1024)
    return [int(x) for x in out[:n]]


def count(board, meta, white):
    b, m = _bm(board, meta)
    return lib().host_count(_p(b), _p(m), int(white))


def count2(board, meta, white):
    b, m = _bm(board, meta)
    return lib().host_count2(_p(b), _p(m), int(white))


def select2(board, meta, white, k):
    b, m = _bm(board, meta)
    return lib().host_select2(_p(b), _p(m), int(white), int(k))


def select_action(board, meta, white, k):
    b, m = _bm(board, meta)
    return lib().host_select_action(_p(b), _p(m), int(white), int(k))


def select(board, meta, white, k):
    b, m = _bm(board, meta)
    return lib().host_select(_p(b), _p(m), int(white), int(k))


def action_legal(board, meta, white, a):
    b, m = _bm(board, meta)
    return bool(lib().host_action_legal(_p(b), _p(m), int(white), int(a)))


def next_state(board, meta, white, action):
    b, m = _bm(board, meta)
    ob = np.zeros(64, dtype=np.int8)
    om = np.zeros(8, dtype=np.uint8)
    rw = ctypes.c_int()
    rc = lib().host_next_state(_p(b), _p(m), int(white), int(action), _p(ob), _p(om), ctypes.byref(rw))
    return rc, ob, om, rw.value


def update_state(board, meta):
    b, m = _bm(board, meta)
    ob = np.zeros(64, dtype=np.int8)
    om = np.zeros(8, dtype=np.uint8)
    lib().host_update_state(_p(b), _p(m), _p(ob), _p(om))
    return ob, om


def perft(board, meta, depth):
    b, m = _bm(board, meta)
    return int(lib().host_perft(_p(b), _p(m), int(depth)))


def perft_small(board, meta, depth):
    b, m = _bm(board, meta)
    return int(lib().host_perft_small(_p(b), _p(m), int(depth)))


def rollout_trace(seed, board_id, plies, init, opponent=0, agent_white=True):
    init = np.ascontiguousarray(init, dtype=np.int8).reshape(64)
    a = np.zeros(plies, dtype=np.int16)
    r = np.zeros(plies, dtype=np.int16)
    d = np.zeros(plies, dtype=np.uint8)
    q = np.zeros(plies, dtype=np.uint8)
    fb = np.zeros(64, dtype=np.int8)
    fm = np.zeros(8, dtype=np.uint8)
    st = np.zeros(8, dtype=np.uint64)
    lib().host_rollout_trace2(_p(init), seed, board_id, plies, int(opponent), int(bool(agent_white)), _p(a), _p(r),
                              _p(d), _p(q), _p(fb), _p(fm), _p(st))
    return dict(action=a, reward=r, done=d, reason=q, final_board=fb, final_meta=fm, stats=st)


class HostEnv:
    def __init__(self, init, opponent=0, agent_white=True, seed=0, board=0):
        self._init = np.ascontiguousarray(init, dtype=np.int8).reshape(64)
        self.h = lib().host_env_new2(_p(self._init), int(opponent), int(bool(agent_white)), int(seed), int(board))

    def pick(self):
        return int(lib().host_env_pick(self.h))

    @property
    def draw(self):
        return int(lib().host_env_draw(self.h))

    def __del__(self):
        if getattr(self, "h", None):
            lib().host_env_free(self.h)

    def reset(self):
        lib().host_env_reset(self.h)

    def step(self, a):
        rw, dn, why = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        rc = lib().host_env_step(self.h, int(a), ctypes.byref(rw), ctypes.byref(dn), ctypes.byref(why))
        return rc, rw.value, dn.value, why.value

    def state(self):
        b = np.zeros(64, dtype=np.int8)
        m = np.zeros(8, dtype=np.uint8)
        lib().host_env_state(self.h, _p(b), _p(m))
        return b, m

    def moves(self):
        out = np.zeros(1024, dtype=np.uint16)
        n = lib().host_env_moves(self.h, _p(out), 1024)
        return [int(x) for x in out[:n]]


# ---- FIDE rules mode (gc_fide.h); meta[7] = en-passant file + 1 ---------------------------
def fide_perft(board, meta, depth):
    b, m = _bm(board, meta)
    return int(lib().host_fide_perft(_p(b), _p(m), int(depth)))


def fide_list(board, meta):
    b, m = _bm(board, meta)
    out = np.zeros(1024, dtype=np.uint16)
    n = lib().host_fide_list(_p(b), _p(m), _p(out), 1024)
    return [int(x) for x in out[:n]]


def fide_rollout(seed, board_id, plies, init):
    init = np.ascontiguousarray(init, dtype=np.int8).reshape(64)
    a = np.zeros(plies, dtype=np.int16)
    r = np.zeros(plies, dtype=np.int16)
    d = np.zeros(plies, dtype=np.uint8)
    q = np.zeros(plies, dtype=np.uint8)
    lib().host_fide_rollout(_p(init), seed, board_id, plies, _p(a), _p(r), _p(d), _p(q))
    return dict(action=a, reward=r, done=d, reason=q)


def mover_checked(board, meta, action):
    """(shortcut, full probe) of the mover's check flag after a legal action (side to move = meta[0])"""
    b, m = _bm(board, meta)
    r = lib().host_mover_checked(_p(b), _p(m), int(action))
    return bool(r & 1), bool(r & 2)


def fide_gen_check(board, meta, depth):
    """None if the shared generator and the per-square walk agree at every node of the FIDE
    perft tree to `depth`; else (board, white, shared count, walk count, ep square) of the first
    node where they differ"""
    b, m = _bm(board, meta)
    ob = np.zeros(64, dtype=np.int8)
    om = np.zeros(8, dtype=np.uint8)
    c = np.zeros(3, dtype=np.int32)
    if lib().host_fide_gen_check(_p(b), _p(m), int(depth), _p(ob), _p(om), _p(c)) == 0:
        return None
    return ob, int(om[0]), int(c[0]), int(c[1]), int(c[2])
