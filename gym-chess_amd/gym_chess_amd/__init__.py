"""gym_chess_amd -- MI355X-native batched chess environment.

Drop-in for the hot path of bobu36000/gym-chess: the PyO3 `ChessEngine`
(/root/reference/src/lib.rs) and ChessEnvV2's reset()/step()/get_possible_moves()
(/root/reference/gym_chess/envs/chess_v2.py), re-built as HIP kernels for gfx950 behind a
C-ABI (include/gymchess.h) bound here with ctypes.
"""
from . import codec  # noqa: F401
from .codec import (  # noqa: F401
    BISHOP_ID,
    BLACK,
    CASTLE_KING_SIDE_BLACK,
    CASTLE_KING_SIDE_WHITE,
    CASTLE_QUEEN_SIDE_BLACK,
    CASTLE_QUEEN_SIDE_WHITE,
    DEFAULT_BOARD,
    KING_ID,
    KNIGHT_ID,
    PAWN_ID,
    QUEEN_ID,
    ROOK_ID,
    WHITE,
)


def __getattr__(name):  # lazy: importing the package must not require a GPU
    if name in ("ChessEngine", "Engine"):
        from . import engine

        return getattr(engine, name)
    if name in ("BatchedChessEnv", "MultiDeviceChessEnv"):
        from . import env

        return getattr(env, name)
    if name in ("ChessEnv",):
        from . import single

        return getattr(single, name)
    raise AttributeError(name)
