"""ChessEngine protocol (lib.rs:1412-1512: dicts + "e2e4" strings) over the C oracle.

Test infrastructure only: lets the CPU suite drive `gym_chess_amd.single.ChessEnv` (which
normally sits on the GPU ChessEngine) against the reference's recorded env traces.
"""
import oracle as O
from gym_chess_amd import codec as C


class OracleChessEngine:
    def next_state(self, state, player, move):
        b, m = C.dict_to_arrays(state)
        rc, nb, nm, rw = O.next_state(b, m, C.player_to_white(player), C.str_to_action(move))
        if rc == -1:
            raise RuntimeError("Bad move - piece is empty !")
        if rc == 1:
            raise SystemError("Both Kings are in check: this position is impossible")
        return C.arrays_to_dict(nb, nm), rw

    def get_possible_moves(self, state, player, attack=False):
        b, m = C.dict_to_arrays(state)
        return [C.action_to_str(x) for x in O.get_possible_moves(b, m, C.player_to_white(player), attack)]

    def get_castle_moves(self, state, player):
        b, m = C.dict_to_arrays(state)
        return [C.action_to_str(x) for x in O.get_castle_moves(b, m, C.player_to_white(player))]

    def update_state(self, state):
        b, m = C.dict_to_arrays(state)
        nb, nm = O.update_state(b, m)
        return C.arrays_to_dict(nb, nm)


class OracleBoard:
    """The single-board op protocol of gym_chess_amd.single.DeviceBoard over the C oracle's
    restatement of chess_v2.py (oracle_single_op): lets the CPU suite (and bench.py's
    configs[0] CPU baseline) run the same ChessEnv without a GPU."""

    def __init__(self, initial_board=None):
        import numpy as np

        from gym_chess_amd.single import _REC

        init = O.DEFAULT_BOARD if initial_board is None else C.board_to_array(initial_board)
        self._e = O.OracleEnv(init, opponent=0, agent_white=True)
        self._rec = np.zeros(1, dtype=_REC)[0]
        self._np = np

    def call(self, op, action=0, flags=0):
        np = self._np
        status, reward, done, reason = self._e.single_op(op, 0 if action is None else action, flags)
        b, m = self._e.state()
        mv = self._e.moves()
        r = self._rec
        r["status"], r["reward"], r["done"], r["reason"] = status, reward, done, reason
        r["env_done"], r["white_to_move"] = int(self._e.done), m[0]
        r["rights"], r["checked"], r["move_count"] = m[1:5], m[5:7], m[7]
        r["board"] = b
        r["nmoves"] = len(mv)
        r["moves"][: len(mv)] = np.array(mv, dtype=np.uint16)
        return r

    def set_state(self, board, flags6):
        """the state setter (oracle_env_set_board): the side to move, move_count, done and the
        window stay -> the record"""
        self._e.set_board(board, flags6)
        return self.call(4)

    def window(self):
        raise NotImplementedError("the oracle keeps every board since reset")

    def close(self):
        pass
