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
