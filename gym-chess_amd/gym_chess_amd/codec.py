"""Encodings shared by the compat engine and the batched env (pure Python, no compute).

Mirrors the reference conventions:
  * piece ids and DEFAULT_BOARD           -- lib.rs:11-17, 41-50; chess_v2.py:17-23, 98-107
  * move strings "e2e4" and castle names  -- lib.rs:36-39, 1278-1290, 1311-1373
  * action ints from*64+to, 4096+castle   -- chess_v2.py:492-532
  * state dict keys                       -- lib.rs:355-395, 1246-1276; chess_v2.py:301-313
"""
import numpy as np

EMPTY_SQUARE_ID = 0
KING_ID = 1
QUEEN_ID = 2
ROOK_ID = 3
BISHOP_ID = 4
KNIGHT_ID = 5
PAWN_ID = 6

WHITE = "WHITE"
BLACK = "BLACK"

CASTLE_KING_SIDE_WHITE = "CASTLE_KING_SIDE_WHITE"
CASTLE_QUEEN_SIDE_WHITE = "CASTLE_QUEEN_SIDE_WHITE"
CASTLE_KING_SIDE_BLACK = "CASTLE_KING_SIDE_BLACK"
CASTLE_QUEEN_SIDE_BLACK = "CASTLE_QUEEN_SIDE_BLACK"
RESIGN = "RESIGN"
CASTLE_MOVES = [
    CASTLE_KING_SIDE_WHITE,
    CASTLE_QUEEN_SIDE_WHITE,
    CASTLE_KING_SIDE_BLACK,
    CASTLE_QUEEN_SIDE_BLACK,
]
# chess_v2.py:497-506
A_KSW, A_QSW, A_KSB, A_QSB, A_RESIGN = 4096, 4097, 4098, 4099, 4100
CASTLE_TO_ACTION = {
    CASTLE_KING_SIDE_WHITE: A_KSW,
    CASTLE_QUEEN_SIDE_WHITE: A_QSW,
    CASTLE_KING_SIDE_BLACK: A_KSB,
    CASTLE_QUEEN_SIDE_BLACK: A_QSB,
}
ACTION_TO_CASTLE = {v: k for k, v in CASTLE_TO_ACTION.items()}
N_ACTIONS = 64 * 64 + 4 + 1  # chess_v2.py:157

DEFAULT_BOARD = [
    [-3, -5, -4, -2, -1, -4, -5, -3],
    [-6, -6, -6, -6, -6, -6, -6, -6],
    [0] * 8,
    [0] * 8,
    [0] * 8,
    [0] * 8,
    [6, 6, 6, 6, 6, 6, 6, 6],
    [3, 5, 4, 2, 1, 4, 5, 3],
]

# Reward constants (chess_v2.py:42-51)
WIN_REWARD = 100
LOSS_REWARD = -100
INVALID_ACTION_REWARD = -10

_COLS = "abcdefgh"


def _action_str(a):
    if a >= 4096:
        return ACTION_TO_CASTLE[a] if a in ACTION_TO_CASTLE else RESIGN
    f, t = divmod(a, 64)
    fr, fc = divmod(f, 8)
    tr, tc = divmod(t, 8)
    return f"{_COLS[fc]}{8 - fr}{_COLS[tc]}{8 - tr}"


_ACTION_STRS = [_action_str(a) for a in range(N_ACTIONS)]  # one lookup per move of a list


def action_to_str(a):
    """action -> reference engine move string (lib.rs:1278-1290 / castle names)."""
    a = int(a)
    return _ACTION_STRS[a] if 0 <= a < N_ACTIONS else _action_str(a)


def actions_to_strs(actions):
    """a move list (uint16 array of engine actions) -> reference move strings"""
    t = _ACTION_STRS
    return [t[a] if a < N_ACTIONS else _action_str(a) for a in actions.tolist()]


def str_to_action(s):
    """reference engine move string -> action (lib.rs:1311-1373)."""
    if s in CASTLE_TO_ACTION:
        return CASTLE_TO_ACTION[s]
    if len(s) != 4 or s[0] not in _COLS or s[2] not in _COLS:
        raise ValueError(f"bad move string {s!r}")
    fr, tr = 8 - int(s[1]), 8 - int(s[3])
    fc, tc = _COLS.index(s[0]), _COLS.index(s[2])
    if not (0 <= fr < 8 and 0 <= tr < 8):
        raise ValueError(f"bad move string {s!r}")
    return (fr * 8 + fc) * 64 + tr * 8 + tc


def action_to_move(a):
    """chess_v2.py:514-531 (as_string=False)."""
    a = int(a)
    if a >= 4096:
        return ACTION_TO_CASTLE.get(a, RESIGN)
    f, t = divmod(a, 64)
    return ((f // 8, f % 8), (t // 8, t % 8))


def move_to_action(m):
    """chess_v2.py:492-506."""
    if isinstance(m, (list, tuple)):
        return (int(m[0][0]) * 8 + int(m[0][1])) * 64 + int(m[1][0]) * 8 + int(m[1][1])
    if m == RESIGN:
        return A_RESIGN
    return CASTLE_TO_ACTION[m]


def rust_move_to_coords(s):
    """chess_v2.py:558-567."""
    if s in CASTLE_MOVES:
        return s
    return action_to_move(str_to_action(s))


def _board_list(board):
    """the common case -- a list of 8 lists of 8 Python ints (the reference's state dicts) --
    without numpy's per-element inference; None when board is anything else"""
    if type(board) is not list or len(board) != 8:
        return None
    flat = []
    for r in board:
        if type(r) is not list or len(r) != 8:
            return None
        flat.extend(r)
    for x in flat:
        if type(x) is not int:
            return None
    if min(flat) < -6 or max(flat) > 6:
        raise ValueError("piece id out of range [-6, 6]")
    return np.array(flat, dtype=np.int8)


def board_to_array(board):
    """list-of-lists / ndarray (8x8, or flat 64) -> int8[64]; raises TypeError like
    convert_py_state."""
    fast = _board_list(board)
    if fast is not None:
        return fast
    a = np.asarray(board)
    if a.shape == (64,):
        a = a.reshape(8, 8)
    if a.shape != (8, 8):
        raise TypeError("board must be 8x8")
    if not np.issubdtype(a.dtype, np.integer):
        raise TypeError("board entries must be integers")
    if a.min() < -6 or a.max() > 6:
        raise ValueError("piece id out of range [-6, 6]")
    return np.ascontiguousarray(a, dtype=np.int8).reshape(64)


def player_to_white(player):
    """lib.rs:424-441: only 'WHITE' / 'BLACK' are valid."""
    if player == WHITE:
        return True
    if player == BLACK:
        return False
    raise ValueError("Invalid Color. Must be 'WHITE' or 'BLACK'")


_STATE_KEYS = (
    "board",
    "current_player",
    "white_king_castle_is_possible",
    "white_queen_castle_is_possible",
    "black_king_castle_is_possible",
    "black_queen_castle_is_possible",
)


def dict_to_arrays(state):
    """convert_py_state (lib.rs:1246-1276) -> (board int8[64], meta uint8[8]).
    Missing key -> KeyError (the reference unwrap()s and panics)."""
    for k in _STATE_KEYS:
        if k not in state:
            raise KeyError(k)
    b = board_to_array(state["board"])
    m = [1 if player_to_white(state["current_player"]) else 0]
    for k in _STATE_KEYS[2:]:
        v = state[k]
        if not isinstance(v, (bool, np.bool_)):
            raise TypeError(f"{k} must be a bool")
        m.append(1 if v else 0)
    return b, np.array(m + [0, 0, 0], dtype=np.uint8)


def arrays_to_dict(board, meta):
    """State::to_py_object (lib.rs:355-395)."""
    m = np.asarray(meta).tolist()
    return {
        "white_king_castle_is_possible": bool(m[1]),
        "white_queen_castle_is_possible": bool(m[2]),
        "black_king_castle_is_possible": bool(m[3]),
        "black_queen_castle_is_possible": bool(m[4]),
        "white_king_is_checked": bool(m[5]),
        "black_king_is_checked": bool(m[6]),
        "board": np.asarray(board).reshape(8, 8).tolist(),  # Python ints
        "current_player": WHITE if m[0] else BLACK,
    }


# compact text form for fixtures: one char per square, white upper-case
_PIECE_CHARS = ".KQRBNP"


def board_to_text(board):
    b = np.asarray(board, dtype=np.int64).reshape(64)
    return "".join(_PIECE_CHARS[v] if v >= 0 else _PIECE_CHARS[-v].lower() for v in b)


def text_to_board(s):
    out = np.zeros(64, dtype=np.int8)
    for i, ch in enumerate(s):
        if ch == ".":
            continue
        v = _PIECE_CHARS.index(ch.upper())
        out[i] = v if ch.isupper() else -v
    return out
