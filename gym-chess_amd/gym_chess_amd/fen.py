"""FEN ingest / export for the reference's state, via the C-ABI's
host-side parser (gc_fen_to_state_rules / gc_state_to_fen_rules; no GPU needed).

Mapping (include/gymchess.h): placement rank 8 first = board row 0 (lib.rs:41-50); side to
move; castling "KQkq" -> white_king / white_queen / black_king / black_queen
*_castle_is_possible (chess_v2.py:301-313); en passant and the half-move clock are ignored
(the reference has neither); full-move number n <-> move_count n - 1.  Under
rules="fide" (gc_fide.h) the en-passant field is kept instead: meta[7] = its file + 1.
"""
import ctypes

import numpy as np

from . import _lib
from . import codec as C

STARTPOS = "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1"


def fen_to_arrays(fen, rules="reference"):
    """-> (board int8[64], meta uint8[8]) with meta = {white_to_move, wkc, wqc, bkc, bqc,
    wchk=0, bchk=0, move_count} (rules="fide": meta[7] = en-passant file + 1, 0 = none).
    Raises GymChessError on a malformed FEN."""
    b = np.zeros(64, dtype=np.int8)
    m = np.zeros(8, dtype=np.uint8)
    _lib.check(_lib.load().gc_fen_to_state_rules(fen.encode(), _lib.ptr(b), _lib.ptr(m), _lib.rules_id(rules)))
    return b, m


def arrays_to_fen(board, meta, rules="reference"):
    b = np.ascontiguousarray(C.board_to_array(board), dtype=np.int8).reshape(64)
    m = np.ascontiguousarray(meta, dtype=np.uint8).reshape(8)
    buf = ctypes.create_string_buffer(128)
    _lib.check(_lib.load().gc_state_to_fen_rules(_lib.ptr(b), _lib.ptr(m), ctypes.cast(buf, ctypes.c_void_p), 128,
                                                 _lib.rules_id(rules)))
    return buf.value.decode()


def fen_to_dict(fen):
    """FEN -> the reference's state dict (check flags False: run ChessEngine.update_state
    to fill them, as chess_v2.py:204 does at reset)."""
    b, m = fen_to_arrays(fen)
    return C.arrays_to_dict(b, m)


def dict_to_fen(state, move_count=0):
    b, m = C.dict_to_arrays(state)
    m[7] = min(int(move_count), 255)
    return arrays_to_fen(b, m)
