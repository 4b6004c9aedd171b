"""Batched ChessEnvV2 on one GPU (chess_v2.py:132-602 semantics).

opponent="none" (each step() is one ply, the caller plays both sides) or "random" (the
device policy replies inside step(), chess_v2.py:275-292); player_color=BLACK makes the
opponent open at every reset (chess_v2.py:208-216).

`BatchedChessEnv(num_boards)` keeps N boards resident in HBM (bitboard SoA) and exposes
the reference env surface vectorised over boards:

    reset(mask=None)            chess_v2.py:183-217
    step(actions)               chess_v2.py:219-294 -> (reward int32[N], done bool[N], reason uint8[N])
    possible_moves / possible_actions / legal_mask / state / board arrays

plus the device-resident random self-play driver of test_benchmark.py
(`step_random`, `rollout`) used by bench.py.

rules="fide" plays FIDE chess (gym-chess_amd/csrc/gc_fide.h) with the
reference env's rewards and bookkeeping; an action promotes to a queen.
"""
import ctypes
import os

import numpy as np

from . import _lib
from . import codec as C

REASONS = {0: "none", 1: "mate", 2: "repetition", 3: "move_cap", 4: "no_moves", 5: "both_kings_checked",
           6: "invalid_action", 7: "already_done", 8: "mated_by_opponent", 9: "opponent_no_move",
           10: "repetition_table_exhausted"}


class BatchedChessEnv:
    def __init__(self, num_boards, device=0, seed=0, initial_board=None, opponent="none", player_color=C.WHITE,
                 rules="reference"):
        self._L = _lib.load()
        self.num_boards = int(num_boards)
        self.device = int(device)
        self.seed = int(seed)
        ib = None
        if initial_board is not None:
            ib = C.board_to_array(initial_board)
        h = ctypes.c_void_p()
        _lib.check(self._L.gc_env_create(self.device, self.num_boards, ctypes.c_uint64(self.seed),
                                         _lib.ptr(ib) if ib is not None else None, ctypes.byref(h)))
        self._h = h
        if opponent not in ("none", "random"):
            raise ValueError(f"Unrecognized opponent policy {opponent} (batched env: 'none' or 'random'; "
                             "drive both sides yourself for a custom opponent)")
        self.opponent = opponent
        self.player_color = player_color
        if opponent != "none" or player_color != C.WHITE:
            _lib.check(self._L.gc_env_set_opponent(self._h, int(opponent == "random"), int(player_color == C.WHITE)))
        self.rules = rules
        if _lib.rules_id(rules):  # FIDE (gc_fide.h): either opponent mode
            _lib.check(self._L.gc_env_set_rules(self._h, _lib.rules_id(rules)))

    def close(self):
        if getattr(self, "_h", None):
            self._L.gc_env_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------ gym surface
    def reset(self, mask=None):
        m = None
        if mask is not None:
            m = np.ascontiguousarray(mask, dtype=np.uint8).reshape(self.num_boards)
        _lib.check(self._L.gc_env_reset(self._h, _lib.ptr(m) if m is not None else None))
        return self.state()

    def step(self, actions):
        a = np.ascontiguousarray(actions, dtype=np.int64).reshape(self.num_boards)
        if (a < 0).any() or (a >= C.N_ACTIONS).any():  # action_space.contains (chess_v2.py:237)
            raise AssertionError(f"ACTION ERROR {a[(a < 0) | (a >= C.N_ACTIONS)][0]}")
        a = a.astype(np.uint16)
        rw = np.zeros(self.num_boards, dtype=np.int32)
        dn = np.zeros(self.num_boards, dtype=np.uint8)
        why = np.zeros(self.num_boards, dtype=np.uint8)
        _lib.check(self._L.gc_env_step(self._h, _lib.ptr(a), _lib.ptr(rw), _lib.ptr(dn), _lib.ptr(why)))
        return rw, dn.astype(bool), why

    def possible_actions(self, cap=320):
        """list of per-board action lists in reference order (chess_v2.py:333-335)."""
        moves, cnt = self.legal_moves(cap)
        return [[int(x) for x in moves[i, : cnt[i]]] for i in range(self.num_boards)]

    def possible_moves(self, cap=320):
        """per-board move lists in the env's coordinate form (chess_v2.py:573-582)."""
        return [[C.action_to_move(a) for a in acts] for acts in self.possible_actions(cap)]

    def legal_moves(self, cap=320):
        moves = np.zeros((self.num_boards, cap), dtype=np.uint16)
        cnt = np.zeros(self.num_boards, dtype=np.int32)
        _lib.check(self._L.gc_env_legal_moves(self._h, _lib.ptr(moves), int(cap), _lib.ptr(cnt)))
        return moves, cnt

    def legal_mask(self):
        """bool[N, 4101] action mask (RL form of possible_actions)."""
        raw = np.zeros((self.num_boards, 65), dtype=np.uint64)
        cnt = np.zeros(self.num_boards, dtype=np.int32)
        _lib.check(self._L.gc_env_legal_mask(self._h, _lib.ptr(raw), _lib.ptr(cnt)))
        bits = np.unpackbits(raw[:, :64].view(np.uint8).reshape(self.num_boards, 64, 8), axis=2, bitorder="little")
        out = np.zeros((self.num_boards, C.N_ACTIONS), dtype=bool)
        out[:, :4096] = bits.reshape(self.num_boards, 4096).astype(bool)
        for c in range(4):
            out[:, 4096 + c] = (raw[:, 64] >> np.uint64(c)) & np.uint64(1) != 0
        return out

    def boards(self):
        b = np.zeros((self.num_boards, 64), dtype=np.int8)
        m = np.zeros((self.num_boards, 8), dtype=np.uint8)
        _lib.check(self._L.gc_env_get_states(self._h, _lib.ptr(b), _lib.ptr(m)))
        return b, m

    def state(self, i=None):
        """state dict(s) in the reference format (chess_v2.py:301-313)."""
        b, m = self.boards()
        if i is not None:
            return C.arrays_to_dict(b[i], m[i])
        return [C.arrays_to_dict(b[k], m[k]) for k in range(self.num_boards)]

    def set_states(self, boards, meta, en_passant=None):
        """boards[i], meta[i] (meta[7] = move_count); repetition windows cleared.  Under
        rules="fide", en_passant = int8[N] files (-1 none) as en_passant() returns them."""
        b = np.ascontiguousarray(boards, dtype=np.int8).reshape(self.num_boards, 64)
        m = np.ascontiguousarray(meta, dtype=np.uint8).reshape(self.num_boards, 8)
        _lib.check(self._L.gc_env_set_states(self._h, _lib.ptr(b), _lib.ptr(m)))
        if en_passant is not None:
            ep = np.ascontiguousarray(en_passant, dtype=np.int8).reshape(self.num_boards)
            _lib.check(self._L.gc_env_set_en_passant(self._h, _lib.ptr(ep)))

    def en_passant(self):
        """int8[N]: en-passant file per board, -1 none (always -1 under the reference's rules)."""
        ep = np.zeros(self.num_boards, dtype=np.int8)
        _lib.check(self._L.gc_env_get_en_passant(self._h, _lib.ptr(ep)))
        return ep

    def set_fens(self, fens):
        """boards[i] := fens[i] (gym_chess_amd.fen mapping); check flags from update_state;
        repetition windows cleared.  Call select_random() before step_random()."""
        if len(fens) != self.num_boards:
            raise ValueError(f"need {self.num_boards} FEN strings, got {len(fens)}")
        arr = (ctypes.c_char_p * self.num_boards)(*[f.encode() for f in fens])
        _lib.check(self._L.gc_env_set_fens(self._h, ctypes.cast(arr, ctypes.c_void_p)))

    def fens(self):
        from .fen import arrays_to_fen

        b, m = self.boards()
        if _lib.rules_id(self.rules):  # FIDE: the en-passant field instead of the move number
            ep = self.en_passant()
            m = m.copy()
            m[:, 7] = np.where(ep < 0, 0, ep + 1).astype(np.uint8)
            return [arrays_to_fen(b[i], m[i], rules=self.rules) for i in range(self.num_boards)]
        return [arrays_to_fen(b[i], m[i]) for i in range(self.num_boards)]

    def observation(self):
        """int8[N, 8, 8] boards (the reference's observation, chess_v2.py:153-158)."""
        return self.boards()[0].reshape(self.num_boards, 8, 8)

    def info(self):
        """the reference's info dict (chess_v2.py:337-353), batched as arrays."""
        b, m = self.boards()
        return dict(move_count=m[:, 7].astype(np.int32), current_player_is_white=m[:, 0].astype(bool),
                    white_king_castle_is_possible=m[:, 1].astype(bool),
                    white_queen_castle_is_possible=m[:, 2].astype(bool),
                    black_king_castle_is_possible=m[:, 3].astype(bool),
                    black_queen_castle_is_possible=m[:, 4].astype(bool),
                    white_king_is_checked=m[:, 5].astype(bool), black_king_is_checked=m[:, 6].astype(bool),
                    white_king_on_the_board=(b == C.KING_ID).any(axis=1),
                    black_king_on_the_board=(b == -C.KING_ID).any(axis=1))

    # ------------------------------------------------------------------ device-resident driver
    def select_random(self):
        _lib.check(self._L.gc_env_select_random(self._h))

    def set_streams(self, k):
        """step_random over k board ranges on k device streams (gc_env_set_streams)."""
        _lib.check(self._L.gc_env_set_streams(self._h, int(k)))

    def paired(self):
        """True when step_random / rollout run the paired two-wave kernels (gc_env_paired)."""
        r = self._L.gc_env_paired(self._h)
        if r < 0:
            _lib.check(r)
        return bool(r)

    def rollout_waves(self):
        """waves per 64 boards of the fused rollout: 4 (quads), 2 (pairs) or 1 (gc_env_rollout_waves)"""
        r = self._L.gc_env_rollout_waves(self._h)
        if r < 0:
            _lib.check(r)
        return int(r)

    def rollout_occ_min_plies(self):
        """the fewest plies per quad launch that run with the window's occupancy filter
        (gc_env_rollout_occ_min_plies; shorter launches probe the table every ply)"""
        return int(self._L.gc_env_rollout_occ_min_plies())

    def step_random(self, n_plies=1):
        _lib.check(self._L.gc_env_step_random(self._h, int(n_plies)))

    def outputs(self):
        n = self.num_boards
        rw = np.zeros(n, dtype=np.int32)
        dn = np.zeros(n, dtype=np.uint8)
        why = np.zeros(n, dtype=np.uint8)
        act = np.zeros(n, dtype=np.uint16)
        ns = np.zeros(n, dtype=np.uint32)
        _lib.check(self._L.gc_env_get_outputs(self._h, _lib.ptr(rw), _lib.ptr(dn), _lib.ptr(why), _lib.ptr(act),
                                              _lib.ptr(ns)))
        return dict(reward=rw, done=dn, reason=why, next_action=act, nsteps=ns)

    def rollout(self, n_plies, trace=False):
        n = self.num_boards
        st = np.zeros(8, dtype=np.uint64)
        if trace:
            ta = np.zeros((n_plies, n), dtype=np.int16)
            tr = np.zeros((n_plies, n), dtype=np.int16)
            td = np.zeros((n_plies, n), dtype=np.uint8)
            tq = np.zeros((n_plies, n), dtype=np.uint8)
            _lib.check(self._L.gc_env_rollout(self._h, int(n_plies), _lib.ptr(ta), _lib.ptr(tr), _lib.ptr(td),
                                              _lib.ptr(tq), _lib.ptr(st)))
            return st, dict(action=ta, reward=tr, done=td, reason=tq)
        _lib.check(self._L.gc_env_rollout(self._h, int(n_plies), None, None, None, None, _lib.ptr(st)))
        return st, None

    def rollout_device(self, n_plies, trace=None, events=(-1, -1)):
        """n_plies env.step() calls of every board under the random self-play policy in one
        launch, asynchronous (gc_env_rollout_device).  trace: None, or a TraceBuffer with room
        for n_plies plies: every ply's outputs land in it on the device.  events: event slots
        recorded right before / after the launches (-1 = none; elapsed_ms reads them)."""
        if trace is not None and trace.plies < n_plies:
            raise ValueError(f"trace buffer holds {trace.plies} plies, need {n_plies}")
        _lib.check(self._L.gc_env_rollout_device(self._h, int(n_plies), trace.ptr if trace is not None else None,
                                                 int(events[0]), int(events[1])))

    def trace_buffer(self, plies):
        """device memory for rollout_device's per-ply outputs ([plies][N] packed words)"""
        return TraceBuffer(self, plies)

    def spill_info(self):
        """the repetition spill table of a BLACK-agent env: dict(bits, used, live)"""
        b = ctypes.c_int()
        u, lv = ctypes.c_uint64(), ctypes.c_uint64()
        _lib.check(self._L.gc_env_spill_info(self._h, ctypes.byref(b), ctypes.byref(u), ctypes.byref(lv)))
        return dict(bits=b.value, used=u.value, live=lv.value)

    def synchronize(self):
        _lib.check(self._L.gc_env_synchronize(self._h))

    def wait_rollout(self):
        """wait for the last rollout_device call's work: its launch's completion word in
        host-mapped memory (quad kernel), else the stream (gc_env_wait_rollout)"""
        _lib.check(self._L.gc_env_wait_rollout(self._h))

    def record_event(self, slot):
        _lib.check(self._L.gc_env_record_event(self._h, int(slot)))

    def elapsed_ms(self, a, b):
        ms = ctypes.c_float()
        _lib.check(self._L.gc_env_elapsed_ms(self._h, int(a), int(b), ctypes.byref(ms)))
        return ms.value

    def window_sum(self):
        v = ctypes.c_uint64()
        _lib.check(self._L.gc_env_window_sum(self._h, ctypes.byref(v)))
        return int(v.value)

    def device_bytes(self):
        return int(self._L.gc_env_device_bytes(self._h))

    # ------------------------------------------------------------------ device-buffer step
    def device_io(self, mask=True, obs=True, count=True, pick=True, select=True, mask_stride=None):
        """Device buffers for step_device (gc_device_alloc on this env's device); with pick and
        select, the pick buffer starts as the random policy's actions for the current states.
        mask_stride: the mask's row stride in words (>= N; None = DeviceIO.default_mask_stride)."""
        return DeviceIO(self, mask=mask, obs=obs, count=count, pick=pick, select=select, mask_stride=mask_stride)

    def step_device(self, io, actions=None, autoreset=False):
        """step() on device buffers (gc_env_step_device), asynchronous on the env's stream.
        actions: a device pointer (int, e.g. a torch tensor's data_ptr()) to uint16[N];
        None = io.pick, the random policy's pick of the previous call (or select_device())."""
        a = io.ptr["pick"] if actions is None else int(actions)
        if not a:
            raise ValueError("no actions: pass a device pointer or allocate io with pick=True")
        p = io.ptr
        _lib.check(self._L.gc_env_step_device2(self._h, a, p["reward"], p["done"], p["reason"], p.get("mask"),
                                               p.get("obs"), p.get("count"), p.get("pick"), int(bool(autoreset)),
                                               io.mask_stride))

    def stream(self):
        """the env's hipStream_t (for callers ordering their own device work with it)"""
        v = ctypes.c_void_p()
        _lib.check(self._L.gc_env_get_stream(self._h, ctypes.byref(v)))
        return v.value

    # ------------------------------------------------------------------ checkpoint / resume
    def checkpoint(self):
        """The whole env as bytes (gc_env_save): states, move counts, done flags, 3-fold
        windows, policy streams, step counters.  load() on an env built with the same
        arguments continues exactly as this one would."""
        need = ctypes.c_uint64()
        _lib.check(self._L.gc_env_checkpoint_bytes(self._h, ctypes.byref(need)))
        buf = np.zeros(need.value, dtype=np.uint8)
        wr = ctypes.c_uint64()
        _lib.check(self._L.gc_env_save(self._h, _lib.ptr(buf), ctypes.c_uint64(buf.size), ctypes.byref(wr)))
        return buf[: wr.value].tobytes()

    def load(self, blob):
        a = np.frombuffer(blob, dtype=np.uint8)
        _lib.check(self._L.gc_env_load(self._h, _lib.ptr(a), ctypes.c_uint64(a.size)))

    def save_to(self, path):
        with open(path, "wb") as f:
            f.write(self.checkpoint())

    def load_from(self, path):
        with open(path, "rb") as f:
            self.load(f.read())


class TraceBuffer:
    """Device trace of rollout_device: one uint64 word per board per ply ([ply][board]):
    action played (int16, -1 = the driver's no-move reset), reward (int16), done, reason."""

    def __init__(self, env, plies):
        self.env = env
        self.plies = int(plies)
        v = ctypes.c_void_p()
        _lib.check(env._L.gc_device_alloc(env.device, ctypes.c_uint64(8 * self.plies * env.num_boards),
                                          ctypes.byref(v)))
        self.ptr = v.value

    def fetch(self, plies=None):
        """host copy of the first `plies` plies as dict(action, reward, done, reason) [ply][board]"""
        w = self.raw(plies)
        return dict(action=(w & np.uint64(0xFFFF)).astype(np.uint16).view(np.int16),
                    reward=((w >> np.uint64(16)) & np.uint64(0xFFFF)).astype(np.uint16).view(np.int16),
                    done=((w >> np.uint64(32)) & np.uint64(0xFF)).astype(np.uint8),
                    reason=((w >> np.uint64(40)) & np.uint64(0xFF)).astype(np.uint8))

    def raw(self, plies=None):
        """host copy of the first `plies` plies as the packed words, uint64 [ply][board]"""
        k = self.plies if plies is None else int(plies)
        w = np.zeros((k, self.env.num_boards), dtype=np.uint64)
        if w.size:
            _lib.check(self.env._L.gc_env_copy(self.env._h, _lib.ptr(w), self.ptr, ctypes.c_uint64(w.nbytes), 2))
        return w

    def close(self):
        if self.ptr:
            self.env._L.gc_device_free(self.env.device, ctypes.c_void_p(self.ptr))
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DeviceIO:
    """Device buffers of one env's step_device outputs: reward i32, done u8, reason u8 and
    optionally mask u64[65][stride] (word-major: word f of board i at f * stride + i, stride >= N),
    obs i8[N][64], count i32, pick u16 (the random policy's next action, which step_device uses
    as the actions when given none).  fetch() copies them to host arrays; upload_actions() fills
    the pick buffer from the host."""

    _SPEC = {"reward": (np.int32, ()), "done": (np.uint8, ()), "reason": (np.uint8, ()),
             "mask": (np.uint64, (65,)), "obs": (np.int8, (64,)), "count": (np.int32, ()), "pick": (np.uint16, ())}

    @staticmethod
    def default_mask_stride(n):
        """From N = 4096 on: N rounded up to a multiple of 512, plus GC_MASK_PAD words (default
        MASK_PAD).  Packed rows of N = 65 536 sit 512 KiB apart and fall on the same HBM
        channels; measured on the quad API step (same box): packed 17.0 us per launch, padded by
        8 words 16.4, by 64 16.2, by 256-4096 15.6-15.8 -- 512 (4 KiB) kept; N = 65 472 packed
        (511.5 KiB apart) 16.8 against 16.2 for 65 536 padded."""
        pad = int(os.environ.get("GC_MASK_PAD", DeviceIO.MASK_PAD))
        return (n + 511) // 512 * 512 + pad if n >= 4096 and pad else n

    MASK_PAD = 512

    def __init__(self, env, mask=True, obs=True, count=True, pick=True, select=True, mask_stride=None):
        self.env = env
        n = env.num_boards
        self.mask_stride = int(self.default_mask_stride(n) if mask_stride is None else mask_stride)
        if self.mask_stride < n:
            raise ValueError(f"mask_stride {self.mask_stride} < num_boards {n}")
        want = {"reward": True, "done": True, "reason": True, "mask": mask, "obs": obs, "count": count, "pick": pick}
        self.ptr = {}
        for k, on in want.items():
            if not on:
                continue
            dt, sh = self._SPEC[k]
            rows = self.mask_stride if k == "mask" else n
            nb = rows * int(np.prod(sh, dtype=np.int64)) * np.dtype(dt).itemsize
            v = ctypes.c_void_p()
            _lib.check(env._L.gc_device_alloc(env.device, ctypes.c_uint64(nb), ctypes.byref(v)))
            self.ptr[k] = v.value
        if pick and select:  # the policy's picks for the current states
            self.select()

    def select(self):
        """pick = the env's current random-policy actions (picked at creation, reset(),
        step_random(), rollout(); after set_states / set_fens call env.select_random() first)"""
        self.upload_actions(self.env.outputs()["next_action"])

    def upload_actions(self, actions):
        a = np.ascontiguousarray(actions, dtype=np.uint16).reshape(self.env.num_boards)
        _lib.check(self.env._L.gc_env_copy(self.env._h, self.ptr["pick"], _lib.ptr(a), ctypes.c_uint64(a.nbytes), 1))

    def fetch(self, *keys):
        """host copies; the mask comes back as [N][65] (the device buffer is word-major
        [65][mask_stride])"""
        out = {}
        n = self.env.num_boards
        for k in keys or self.ptr:
            dt, sh = self._SPEC[k]
            shape = (65, self.mask_stride) if k == "mask" else (n,) + sh
            a = np.zeros(shape, dtype=dt)
            _lib.check(self.env._L.gc_env_copy(self.env._h, _lib.ptr(a), self.ptr[k], ctypes.c_uint64(a.nbytes), 2))
            out[k] = np.ascontiguousarray(a[:, :n].T) if k == "mask" else a
        return out

    def close(self):
        for v in self.ptr.values():
            self.env._L.gc_device_free(self.env.device, ctypes.c_void_p(v))
        self.ptr = {}

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class MultiDeviceChessEnv:
    """`device_ids` form of the batched env (SURVEY.md §5 Config, §8e): num_boards boards per
    device, one BatchedChessEnv per device, global board g on device g // num_boards.  Device
    calls run in one host thread per device (ctypes releases the GIL), no collective; the
    policy stream of replica r is keyed seed + (r << 40) (gym_chess_amd.replicas)."""

    def __init__(self, num_boards, device_ids=(0,), seed=0, **kw):
        from .replicas import Replicas

        # one thread per device in THIS process, even inside a launched (torchrun) job: the
        # device_ids contract does not depend on WORLD_SIZE
        self.rep = Replicas(gpus=len(device_ids), devices=device_ids, mode="threads")
        self.num_boards = int(num_boards)
        self.envs = self.rep.run(lambda rp: BatchedChessEnv(num_boards, device=rp.device, seed=rp.board_seed(seed), **kw))

    @property
    def total_boards(self):
        return self.num_boards * len(self.envs)

    def _each(self, fn):
        return self.rep.run(lambda rp: fn(self.envs[self.rep.local.index(rp)]))

    def _split(self, x):
        x = np.asarray(x)
        return [x[k * self.num_boards:(k + 1) * self.num_boards] for k in range(len(self.envs))]

    def reset(self, mask=None):
        parts = self._split(mask) if mask is not None else [None] * len(self.envs)
        self.rep.run(lambda rp: self.envs[self.rep.local.index(rp)].reset(parts[self.rep.local.index(rp)]))

    def step(self, actions):
        parts = self._split(actions)
        out = self.rep.run(lambda rp: self.envs[self.rep.local.index(rp)].step(parts[self.rep.local.index(rp)]))
        return tuple(np.concatenate([o[k] for o in out]) for k in range(3))

    def set_streams(self, k):
        """step_random over k board ranges on k device streams, on every device"""
        self._each(lambda e: e.set_streams(k))

    def step_random(self, n_plies=1):
        self._each(lambda e: e.step_random(n_plies))

    def rollout(self, n_plies):
        """fused random self-play on every device; stats8 summed over devices"""
        st = self._each(lambda e: e.rollout(n_plies)[0])
        return np.sum(st, axis=0, dtype=np.uint64)

    def boards(self):
        out = self._each(lambda e: e.boards())
        return np.concatenate([o[0] for o in out]), np.concatenate([o[1] for o in out])

    def outputs(self):
        out = self._each(lambda e: e.outputs())
        return {k: np.concatenate([o[k] for o in out]) for k in out[0]}

    def synchronize(self):
        self._each(lambda e: e.synchronize())

    def close(self):
        for e in getattr(self, "envs", []):
            e.close()
        self.envs = []

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
