"""Single-board ChessEnvV2 on the device.

`ChessEnv` has the surface of the reference's `ChessEnvV2`
(/root/reference/gym_chess/envs/chess_v2.py:132-602), so user code written against the
reference env runs unchanged:

    env = ChessEnv(player_color="WHITE", opponent="random", log=False)
    state = env.reset()
    state, reward, done, info = env.step(action)

The env's bookkeeping -- validation, the done / move-cap early returns, player_move with
the 3-fold count of the PRE-move board (Q8), rewards, mate, the move count, the BLACK
opening -- runs on the device, in the batched env's step code (gc_env.h), on one board of a
gc_env: each step() is ONE launch (gc_env_single_call) whose result (state, outputs and the
next move list in reference order) lands in a host-mapped record -- no copy, no second
copy of chess_v2.py here.  Only the opponent policy runs on the host, as in the reference:
a callable, or "random" = numpy's GLOBAL generator over the move list (116-127), so a seeded
driver replays the reference's games move for move; a step with an opponent is split where
the policy must see the list (AGENT, then REPLY: two launches).  With no legal move the
random policy returns "resign", which maps to no action and fails in action_to_move
(TypeError), and the engine's both-kings-checked error raises SystemError (lib.rs:1442-1446),
both as in the reference.

saved_boards is the reference's dict (chess_v2.py:192, 404-405: every pre-move board since
reset, keyed by encode_board's string) kept on the host beside the device's 3-fold window
(device_window(): the boards since the last pawn move or capture, the only ones that can
recur, with which the device decides the 3-fold end).  Assigning env.state (315-323) changes
the board and the six flags only: the side to move, move_count, done, saved_boards and the
device window stay, and possible_moves stays the list of the board before, as in the
reference -- the next step() validates against it.

Differences: action_to_move_str returns the move string (the reference's version references
an undefined name, chess_v2.py:532); a state dict missing a flag sets it False (the reference
stores None, which its engine then rejects); after a state assignment, an action that the
stale list holds but the new board does not allow raises NotImplementedError (the reference
would apply it unchecked through next_state, lib.rs:679-784).

`backend=` takes any object with the single-board op protocol (`call(op, action, flags)` ->
record); the tests plug in the CPU oracle's restatement to check this class without a GPU.
`engine` (lazily a ChessEngine on the same device) serves the stateless helpers
get_possible_moves / get_castle_moves / next_state with explicit states.
"""
import struct
import sys
from collections import defaultdict
from io import StringIO

import numpy as np

from . import codec as C
from .codec import (BLACK, CASTLE_KING_SIDE_BLACK, CASTLE_KING_SIDE_WHITE, CASTLE_MOVES, CASTLE_QUEEN_SIDE_BLACK,
                    CASTLE_QUEEN_SIDE_WHITE, DEFAULT_BOARD, INVALID_ACTION_REWARD, KING_ID, LOSS_REWARD, RESIGN, WHITE,
                    WIN_REWARD)

MOVES_MAX = 149  # chess_v2.py:141
_ENCODE = "0ABCDEFfedcba"  # chess_v2.py:600: piece id -> character (negative ids from the end)
_ENC_TABLE = bytes(ord(_ENCODE[(b if b < 128 else b - 256)]) if (b < 7 or b > 249) else 63 for b in range(256))

# chess_v2.py:64-84 (icons and descriptions by piece id)
_ICON = {-6: "♙", -5: "♘", -4: "♗", -3: "♖", -2: "♕", -1: "♔", 0: ".",
         1: "♚", 2: "♛", 3: "♜", 4: "♝", 5: "♞", 6: "♟"}
_DESC = {0: "", 1: "K", 2: "Q", 3: "R", 4: "B", 5: "N", 6: ""}
_ANSI_FG = {"gray": 30, "red": 31, "green": 32, "yellow": 33, "blue": 34, "magenta": 35, "cyan": 36, "white": 37,
            "crimson": 38}


def _colorize(s, color, highlight=False):  # gym.utils.colorize
    code = _ANSI_FG[color] + (10 if highlight else 0)
    return f"\x1b[{code}m{s}\x1b[0m"


def highlight(string, background="white", color="gray"):
    return _colorize(_colorize(string, color), background, highlight=True)


class Discrete:
    """spaces.Discrete(n) subset used by the env (contains / n / sample)."""

    def __init__(self, n):
        self.n = int(n)

    def contains(self, x):
        if isinstance(x, (int, np.integer)) and not isinstance(x, bool):
            return 0 <= int(x) < self.n
        if isinstance(x, np.ndarray) and x.shape == () and x.dtype.kind in "iu":
            return 0 <= int(x) < self.n
        return False

    def sample(self):
        return int(np.random.randint(self.n))


class Box:
    def __init__(self, low, high, shape):
        self.low, self.high, self.shape = low, high, tuple(shape)


def make_random_policy(np_random, bot_player):
    """chess_v2.py:116-127: uniform over env.possible_moves with numpy's global generator."""

    def random_policy(env):
        moves = env.possible_moves
        if len(moves) == 0:
            return "resign"
        return moves[np.random.choice(np.arange(len(moves)))]

    return random_policy


OP_RESET, OP_AGENT, OP_REPLY, OP_OPEN, OP_SYNC = 0, 1, 2, 3, 4  # gc_env_single_call ops
R_REPETITION, R_INVALID, R_DONE_ALREADY, R_MOVE_CAP = 2, 6, 7, 3  # reason codes (env.REASONS)
_BOTH_CHECKED = "Both Kings are in check: this position is impossible"  # lib.rs:1442-1446


class DeviceBoard:
    """One board of a gc_env driven by gc_env_single_call: the env's step bookkeeping on the
    device, its result read from the host-mapped gc_single_record."""

    def __init__(self, initial_board, agent_white, device=0):
        import ctypes

        from . import _lib

        self._ct = ctypes
        self._L = _lib.load()
        self._check = _lib.check
        ib = C.board_to_array(initial_board)
        h = ctypes.c_void_p()
        self._check(self._L.gc_env_create(int(device), 1, ctypes.c_uint64(0), _lib.ptr(ib), ctypes.byref(h)))
        self._h = h
        self._check(self._L.gc_env_single_setup(self._h, int(bool(agent_white))))
        self._rec = ctypes.c_void_p()
        self._view = None

    def call(self, op, action=0, flags=0):
        self._check(self._L.gc_env_single_call(self._h, 0, int(op), int(action), int(flags), self._ct.byref(self._rec)))
        return self._mapped()

    def _mapped(self):
        """the host-mapped record (its address is fixed per env) as a memoryview"""
        if self._view is None:
            self._view = memoryview((self._ct.c_uint8 * _REC.itemsize).from_address(self._rec.value))
        return self._view

    def set_state(self, board, flags6):
        """the state setter: board int8[64], flags6 = the 4 rights + 2 check flags; the side to
        move, move_count, done and the window stay (gc_env_single_set) -> the record"""
        b = np.ascontiguousarray(board, dtype=np.int8).reshape(64)
        f = np.ascontiguousarray(flags6, dtype=np.uint8).reshape(6)
        self._check(self._L.gc_env_single_set(self._h, 0, b.ctypes.data_as(self._ct.c_void_p),
                                              f.ctypes.data_as(self._ct.c_void_p), self._ct.byref(self._rec)))
        return self._mapped()

    def window(self):
        """the live 3-fold window: {board bytes: count}"""
        ct = self._ct
        n = ct.c_int()
        self._check(self._L.gc_env_window_boards(self._h, 0, None, None, 0, ct.byref(n)))
        b = np.zeros((max(n.value, 1), 64), dtype=np.int8)
        c = np.zeros(max(n.value, 1), dtype=np.uint8)
        self._check(self._L.gc_env_window_boards(self._h, 0, b.ctypes.data_as(ct.c_void_p), c.ctypes.data_as(ct.c_void_p),
                                                 n.value, ct.byref(n)))
        return {b[k].tobytes(): int(c[k]) for k in range(n.value)}

    def close(self):
        if getattr(self, "_h", None):
            self._L.gc_env_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# gc_single_record (include/gymchess.h)
_REC = np.dtype([("status", "<i4"), ("reward", "<i4"), ("done", "u1"), ("reason", "u1"), ("env_done", "u1"),
                 ("white_to_move", "u1"), ("rights", "u1", (4,)), ("checked", "u1", (2,)), ("move_count", "<u2"),
                 ("nmoves", "<i4"), ("board", "i1", (64,)), ("moves", "<u2", (320,))])
assert _REC.itemsize == 728  # = sizeof(gc_single_record), static_assert in gymchess.hip
_HDR = struct.Struct("<iiBBBB4B2BHi")  # the record's fields before the board (_REC's layout)
_BOARD_AT = _REC.fields["board"][1]
_MOVES_AT = _REC.fields["moves"][1]
assert _HDR.size == _BOARD_AT
_ROWS = [struct.Struct("8b")] * 8

GC_SINGLE_MOVES_CAP = 320
_ACTION_MOVE = [C.action_to_move(a) if a < 4096 else C.ACTION_TO_CASTLE.get(a) for a in range(C.N_ACTIONS - 1)]


class ChessEnv:
    metadata = {"render.modes": ["human", "string"]}

    def __init__(self, player_color=WHITE, opponent="random", log=True, initial_board=DEFAULT_BOARD, device=0,
                 backend=None, engine=None):
        self.moves_max = MOVES_MAX
        self.log = log
        self.initial_board = initial_board
        self.device = device
        self._engine = engine
        self.observation_space = Box(-6, 6, (8, 8))
        self.action_space = Discrete(C.N_ACTIONS)
        self.player = player_color
        self.player_2 = self.get_other_player(player_color)
        self.opponent = opponent
        self.seed()
        self._b = backend if backend is not None else DeviceBoard(initial_board, player_color == WHITE, device)
        self.reset()

    @property
    def engine(self):
        """the stateless engine of the explicit-state helpers (chess_v2.py:146)"""
        if self._engine is None:
            from .engine import ChessEngine

            self._engine = ChessEngine(self.device)
        return self._engine

    # ---------------------------------------------------------------- lifecycle
    def seed(self, seed=None):
        self.np_random = np.random.RandomState(seed)
        if isinstance(self.opponent, str):
            if self.opponent == "random":
                self.opponent_policy = make_random_policy(self.np_random, self.player_2)
            elif self.opponent == "none":
                self.opponent_policy = None
            else:
                raise ValueError(f"Unrecognized opponent policy {self.opponent}")
        else:
            self.opponent_policy = self.opponent
        return [seed]

    def _take(self, rec):
        """mirror the device record (a buffer in gc_single_record's layout: the host-mapped
        record itself, or a numpy record): state, side to move, done, move count, move list;
        returns {status, reward, reason}"""
        if isinstance(rec, np.void):
            rec = rec.tobytes()
        (status, reward, _, reason, env_done, wtm, r0, r1, r2, r3, c0, c1, mc, n) = _HDR.unpack_from(rec)
        if status:
            print(_BOTH_CHECKED)
            raise SystemError(_BOTH_CHECKED)
        bb = bytes(rec[_BOARD_AT:_BOARD_AT + 64])
        self.board = [list(_ROWS[0].unpack_from(bb, 8 * r)) for r in range(8)]
        self._key = bb.translate(_ENC_TABLE).decode("ascii")  # encode_board of it
        self.white_king_castle_is_possible, self.white_queen_castle_is_possible = bool(r0), bool(r1)
        self.black_king_castle_is_possible, self.black_queen_castle_is_possible = bool(r2), bool(r3)
        self.white_king_is_checked, self.black_king_is_checked = bool(c0), bool(c1)
        self.current_player = WHITE if wtm else BLACK
        self.done = bool(env_done)
        self.move_count = mc
        if n > GC_SINGLE_MOVES_CAP:
            raise RuntimeError(f"{n} legal moves: more than the record holds")
        am = _ACTION_MOVE
        self._possible_moves = [am[a] for a in struct.unpack_from(f"<{n}H", rec, _MOVES_AT)]
        return {"status": status, "reward": reward, "reason": reason}

    def _ply(self, op, action, flags=0):
        """one player_move on the device; with log, the reference's print + render of the
        pre-move board (chess_v2.py:409-411, skipped when the move ends by 3-fold)"""
        if op != OP_AGENT and action is None:
            self.action_to_move(action)  # the random policy's "resign": TypeError, as the reference
        mover, pre, key = self.current_player, self.board, self._key
        stale = self._stale
        rec = self._take(self._b.call(op, action, flags))
        if stale and rec["reason"] == R_INVALID:
            raise NotImplementedError(
                f"action {action} is in possible_moves from before the state assignment but not legal on the "
                "assigned board: the reference would apply it unchecked (next_state, lib.rs:679-784)")
        self._stale = False
        if rec["reason"] not in (R_INVALID, R_DONE_ALREADY, R_MOVE_CAP):
            self._saved[key] += 1  # player_move ran (chess_v2.py:404-405)
        if self.log and rec["reason"] not in (R_INVALID, R_DONE_ALREADY, R_MOVE_CAP, R_REPETITION):
            board, self.board = self.board, pre
            print(" " * 10, ">" * 10, mover)
            self.render_moves([self.action_to_move(action)], mode="human")
            self.board = board
        return rec

    def reset(self):
        self.repetitions = 0
        self._saved = defaultdict(int)  # saved_boards (chess_v2.py:192)
        self._stale = False
        self.white_king_on_the_board = self.piece_is_on_board(self.initial_board, KING_ID)
        self.black_king_on_the_board = self.piece_is_on_board(self.initial_board, -KING_ID)
        self._take(self._b.call(OP_RESET))
        if self.player == BLACK:  # the opponent opens as WHITE (chess_v2.py:208-216)
            self._ply(OP_OPEN, self.move_to_action(self.opponent_policy(self)))
        return self.state

    def step(self, action):
        assert self.action_space.contains(action), "ACTION ERROR {}".format(action)
        if self._stale:  # after a state assignment: 239-258 against the stale list and done
            if action not in self.possible_actions:
                return self.state, INVALID_ACTION_REWARD, self.done, self.info
            if self.done or self.move_count > self.moves_max:
                return self.state, 0.0, True, self.info
        opp = self.opponent_policy is not None
        rec = self._ply(OP_AGENT, int(action), 1 if opp else 0)
        why = int(rec["reason"])
        if why == R_INVALID:  # 239-242
            return self.state, INVALID_ACTION_REWARD, self.done, self.info
        if why in (R_DONE_ALREADY, R_MOVE_CAP):  # 245-258
            return self.state, 0.0, True, self.info
        reward = int(rec["reward"])
        if self.done or not opp:
            return self.state, reward, self.done, self.info
        rec = self._ply(OP_REPLY, self.move_to_action(self.opponent_policy(self)))  # 275-288
        return self.state, reward + int(rec["reward"]), self.done, self.info

    def close(self):
        self._b.close()

    # ---------------------------------------------------------------- state
    def switch_player(self):
        self.current_player = self.get_other_player(self.current_player)
        return self.current_player

    @property
    def state(self):
        return dict(
            board=self.board,
            current_player=self.current_player,
            white_king_castle_is_possible=self.white_king_castle_is_possible,
            white_queen_castle_is_possible=self.white_queen_castle_is_possible,
            black_king_castle_is_possible=self.black_king_castle_is_possible,
            black_queen_castle_is_possible=self.black_queen_castle_is_possible,
            white_king_is_checked=self.white_king_is_checked,
            black_king_is_checked=self.black_king_is_checked,
        )

    @state.setter
    def state(self, state):  # chess_v2.py:315-323: the board and the six flags only
        if not hasattr(self._b, "set_state"):
            raise NotImplementedError("this backend cannot take a state")
        flags = [bool(state.get(k)) for k in ("white_king_castle_is_possible", "white_queen_castle_is_possible",
                                              "black_king_castle_is_possible", "black_queen_castle_is_possible",
                                              "white_king_is_checked", "black_king_is_checked")]
        moves, done = self._possible_moves, self.done
        self._take(self._b.set_state(C.board_to_array(state.get("board")), np.array(flags, dtype=np.uint8)))
        self._possible_moves, self.done = moves, done  # the reference's possible_moves stay until a move
        self._stale = True

    @property
    def saved_boards(self):
        """chess_v2.py's saved_boards: {encode_board(): pre-move occurrences} of every
        player_move since reset (the device decides the 3-fold end from its own window)"""
        return self._saved

    def device_window(self):
        """the device's live 3-fold window {board bytes: pre-move occurrences}: the boards since
        the last pawn move or capture"""
        return self._b.window()

    @property
    def possible_moves(self):
        return self._possible_moves

    @possible_moves.setter
    def possible_moves(self, moves):
        self._possible_moves = moves

    @property
    def possible_actions(self):
        return [self.move_to_action(m) for m in self.possible_moves]

    @property
    def info(self):
        return dict(
            move_count=self.move_count,
            current_player=self.current_player,
            possible_moves=self.possible_moves,
            white_king_castle_is_possible=self.white_king_castle_is_possible,
            white_queen_castle_is_possible=self.white_queen_castle_is_possible,
            black_king_castle_is_possible=self.black_king_castle_is_possible,
            black_queen_castle_is_possible=self.black_queen_castle_is_possible,
            white_king_is_checked=self.white_king_is_checked,
            black_king_is_checked=self.black_king_is_checked,
            white_king_on_the_board=self.white_king_on_the_board,
            black_king_on_the_board=self.black_king_on_the_board,
        )

    @property
    def opponent_player(self):
        return BLACK if self.current_player == WHITE else WHITE

    @property
    def current_player_is_white(self):
        return self.current_player == WHITE

    @property
    def current_player_is_black(self):
        return not self.current_player_is_white

    def king_is_checked(self, player):
        return self.white_king_is_checked if player == WHITE else self.black_king_is_checked

    @staticmethod
    def piece_is_on_board(board, piece_id):
        return bool((np.asarray(board).reshape(64) == piece_id).any())

    def player_can_castle(self, player):  # AND of the two rights, as the reference has it
        if player == WHITE:
            return self.white_king_castle_is_possible and self.white_queen_castle_is_possible
        return self.black_king_castle_is_possible and self.black_queen_castle_is_possible

    @staticmethod
    def get_other_player(player):
        return BLACK if player == WHITE else WHITE

    def next_state(self, state, player, move):
        """the engine's next_state of an explicit state (no env change)"""
        if state is None:
            state = self.state
        return self.engine.next_state(state, player, self.move_to_str_code(move))

    def encode_board(self):  # chess_v2.py:599-602
        return np.asarray(self.board, dtype=np.int8).reshape(64).tobytes().translate(_ENC_TABLE).decode("ascii")

    # ---------------------------------------------------------------- moves
    def get_possible_actions(self):
        return [self.move_to_action(m) for m in self.get_possible_moves(player=self.current_player)]

    def get_possible_moves(self, state=None, player=None, attack=False):
        if state is None:
            state = self.state
        if player is None:
            player = self.current_player
        return [self.rust_move_to_coords(m) for m in self.engine.get_possible_moves(state, player, attack)]

    def get_castle_moves(self, state=None, player=None):
        if state is None:
            state = self.state
        if player is None:
            player = self.current_player
        return [self.rust_move_to_coords(m) for m in self.engine.get_castle_moves(state, player)]

    def is_resignation(self, action):  # never: chess_v2.py:596-597
        return False

    @staticmethod
    def move_to_action(move):
        if type(move) in (list, tuple):
            return (move[0][0] * 8 + move[0][1]) * 64 + move[1][0] * 8 + move[1][1]
        if move in C.CASTLE_TO_ACTION:
            return C.CASTLE_TO_ACTION[move]
        if move == RESIGN:
            return C.A_RESIGN
        return None  # e.g. the random policy's "resign" (lower case): no action

    def action_to_move(self, action):
        if action >= 64 * 64:
            return C.ACTION_TO_CASTLE.get(action, RESIGN if action == C.A_RESIGN else None)
        return ((action // 64 // 8, action // 64 % 8), (action % 64 // 8, action % 64 % 8))

    def action_to_move_str(self, action):
        return self.move_to_str_code(self.action_to_move(action))

    @staticmethod
    def move_to_str_code(move):
        if move in CASTLE_MOVES:
            return move
        (x0, y0), (x1, y1) = move
        return f"{'abcdefgh'[y0]}{8 - x0}{'abcdefgh'[y1]}{8 - x1}"

    def move_to_string(self, move):
        if move in (CASTLE_KING_SIDE_WHITE, CASTLE_KING_SIDE_BLACK):
            return "O-O"
        if move in (CASTLE_QUEEN_SIDE_WHITE, CASTLE_QUEEN_SIDE_BLACK):
            return "O-O-O"
        (x0, y0), (x1, y1) = move
        b = np.asarray(self.board).reshape(8, 8)
        desc = _DESC[abs(int(b[x0, y0]))]
        cap = "x" if b[x1, y1] != 0 else ""
        return f"{desc}{'abcdefgh'[y0]}{8 - x0}{cap}{'abcdefgh'[y1]}{8 - x1}"

    @staticmethod
    def rust_move_to_coords(move):
        if move in CASTLE_MOVES:
            return move
        return C.action_to_move(C.str_to_action(move))

    # ---------------------------------------------------------------- rendering
    def board_to_grid(self):
        return [[f" {_ICON[int(sq)]} " for sq in row] for row in np.asarray(self.board).reshape(8, 8)]

    @staticmethod
    def render_grid(grid, mode="human"):
        out = sys.stdout if mode == "human" else StringIO()
        out.write("    " + "-" * 25 + "\n")
        for i, row in enumerate(grid):
            out.write(f" {8 - i} | " + "".join(row) + "|\n")
        out.write("    " + "-" * 25 + "\n      a  b  c  d  e  f  g  h \n")
        if mode == "string":
            return out.getvalue()
        if mode != "human":
            return out

    def render(self, mode="human"):
        return self.render_grid(self.board_to_grid(), mode=mode)

    def render_moves(self, moves, mode="human"):
        grid = self.board_to_grid()
        b = np.asarray(self.board).reshape(8, 8)
        castle_cells = {
            CASTLE_QUEEN_SIDE_WHITE: (7, [0, 4], [(1, " >>"), (2, "> <"), (3, "<< ")]),
            CASTLE_KING_SIDE_WHITE: (7, [4, 7], [(5, " >>"), (6, "<< ")]),
            CASTLE_QUEEN_SIDE_BLACK: (0, [0, 4], [(1, " >>"), (2, "> <"), (3, "<< ")]),
            CASTLE_KING_SIDE_BLACK: (0, [4, 7], [(5, " >>"), (6, "<< ")]),
        }
        for move in moves:
            if isinstance(move, str) and move in castle_cells:
                r, ends, arrows = castle_cells[move]
                for c in ends:
                    grid[r][c] = highlight(grid[r][c], background="white")
                for c, s in arrows:
                    grid[r][c] = highlight(s, background="green")
                continue
            (x0, y0), (x1, y1) = move
            if len(grid[x0][y0]) < 4:
                grid[x0][y0] = highlight(grid[x0][y0], background="white")
            if len(grid[x1][y1]) < 4:
                grid[x1][y1] = highlight(grid[x1][y1], background="red" if b[x1, y1] else "green")
        return self.render_grid(grid, mode=mode)
