"""Single-board ChessEnvV2 on the GPU engine.

`ChessEnv` is the reference's `ChessEnvV2` (/root/reference/gym_chess/envs/chess_v2.py:132-602)
re-stated over this package's `ChessEngine` (one gc_engine_* launch per engine call), so
user code written against the reference env runs unchanged:

    env = ChessEnv(player_color="WHITE", opponent="random", log=False)
    state = env.reset()
    state, reward, done, info = env.step(action)

Behaviour kept from the reference, including its quirks:
  * step(): invalid action -> INVALID_ACTION_REWARD with the state unchanged, checked before
    `done` (chess_v2.py:239-242); done / move_count > 149 -> (state, 0.0, True, info)
    (245-258); a valid move scores -10 + the captured value (261-264); opponent mated ->
    +100 (269-272); with an opponent, -opp_reward and -100 when the agent is mated
    (275-288); move_count advances when WHITE is to move after the step (291-292).
  * 3-fold repetition counts the PRE-move board only (player_move, 393-412: Q8).
  * reset() with player_color=BLACK lets the opponent open as WHITE (208-216).
  * the "random" opponent draws with numpy's GLOBAL generator (`np.random.choice` over the
    move list, 116-127), so a seeded driver reproduces the reference's games move for move;
    with no legal move it returns "resign", which maps to no action and fails in
    action_to_move (TypeError), as in the reference.
  * the engine raises SystemError when both kings end up in check (lib.rs:1442-1446).
Deliberate difference: action_to_move_str returns the move string (the reference's
version references an undefined name, chess_v2.py:532).

`engine=` accepts any object with the ChessEngine protocol (the tests plug in the CPU
oracle to check this class itself on a machine without a GPU).
"""
import sys
from io import StringIO

import numpy as np

from . import codec as C
from .codec import (BLACK, CASTLE_KING_SIDE_BLACK, CASTLE_KING_SIDE_WHITE, CASTLE_MOVES, CASTLE_QUEEN_SIDE_BLACK,
                    CASTLE_QUEEN_SIDE_WHITE, DEFAULT_BOARD, INVALID_ACTION_REWARD, KING_ID, LOSS_REWARD, RESIGN, WHITE,
                    WIN_REWARD)

MOVES_MAX = 149  # chess_v2.py:141

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


class ChessEnv:
    metadata = {"render.modes": ["human", "string"]}

    def __init__(self, player_color=WHITE, opponent="random", log=True, initial_board=DEFAULT_BOARD, device=0,
                 engine=None):
        self.moves_max = MOVES_MAX
        self.log = log
        self.initial_board = initial_board
        if engine is None:
            from .engine import ChessEngine

            engine = ChessEngine(device)
        self.engine = engine
        self.observation_space = Box(-6, 6, (8, 8))
        self.action_space = Discrete(C.N_ACTIONS)
        self.player = player_color
        self.player_2 = self.get_other_player(player_color)
        self.opponent = opponent
        self.seed()
        self.reset()

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

    def reset(self):
        self.board = self.initial_board
        self.done = False
        self.current_player = WHITE
        self.saved_boards = {}
        self.repetitions = 0
        self.move_count = 0
        self.white_king_castle_is_possible = True
        self.white_queen_castle_is_possible = True
        self.black_king_castle_is_possible = True
        self.black_queen_castle_is_possible = True
        self.white_king_is_checked = False
        self.black_king_is_checked = False
        self.white_king_on_the_board = self.piece_is_on_board(self.board, KING_ID)
        self.black_king_on_the_board = self.piece_is_on_board(self.board, -KING_ID)
        self.state = self.engine.update_state(self.state)
        self.possible_moves = self.get_possible_moves(state=self.state, player=WHITE)
        if self.player == BLACK:  # the opponent opens as WHITE (chess_v2.py:208-216)
            first = self.move_to_action(self.opponent_policy(self))
            self.state, _, _ = self.player_move(first)
            self.move_count += 1
            self.current_player = BLACK
            self.possible_moves = self.get_possible_moves(state=self.state, player=BLACK)
        return self.state

    def step(self, action):
        assert self.action_space.contains(action), "ACTION ERROR {}".format(action)
        if action not in self.possible_actions:
            return self.state, INVALID_ACTION_REWARD, self.done, self.info
        if self.done:
            return self.state, 0.0, True, self.info
        if self.move_count > self.moves_max:
            return self.state, 0.0, True, self.info
        reward = INVALID_ACTION_REWARD
        self.state, move_reward, self.done = self.player_move(action)
        reward += move_reward
        other = self.switch_player()
        self.possible_moves = self.get_possible_moves(player=other)
        if not self.possible_moves and self.king_is_checked(player=other):
            self.done = True
            reward += WIN_REWARD
        if self.done:
            return self.state, reward, self.done, self.info
        if self.opponent_policy:
            opp_action = self.move_to_action(self.opponent_policy(self))
            self.state, opp_reward, self.done = self.player_move(opp_action)
            agent = self.switch_player()
            self.possible_moves = self.get_possible_moves(player=agent)
            reward -= opp_reward
            if not self.possible_moves and self.king_is_checked(player=agent):
                self.done = True
                reward += LOSS_REWARD
        if self.current_player == WHITE:
            self.move_count += 1
        return self.state, reward, self.done, self.info

    def close(self):
        pass

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
    def state(self, state):  # current_player is NOT taken from the dict (chess_v2.py:316-324)
        self.board = state.get("board")
        self.white_king_castle_is_possible = state.get("white_king_castle_is_possible")
        self.white_queen_castle_is_possible = state.get("white_queen_castle_is_possible")
        self.black_king_castle_is_possible = state.get("black_king_castle_is_possible")
        self.black_queen_castle_is_possible = state.get("black_queen_castle_is_possible")
        self.white_king_is_checked = state.get("white_king_is_checked")
        self.black_king_is_checked = state.get("black_king_is_checked")

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

    def player_move(self, action):
        """-> (state, reward, done); the PRE-move board feeds the 3-fold count."""
        if self.is_resignation(action):
            return self.state, LOSS_REWARD, True
        move = self.action_to_move(action)
        new_state, reward = self.next_state(self.state, self.current_player, move)
        key = self.encode_board()
        self.saved_boards[key] = self.saved_boards.get(key, 0) + 1
        if self.saved_boards[key] >= 3:
            return new_state, reward, True
        if self.log:
            print(" " * 10, ">" * 10, self.current_player)
            self.render_moves([move], mode="human")
        return new_state, reward, False

    def next_state(self, state, player, move):
        if state is None:
            state = self.state
        return self.engine.next_state(state, player, self.move_to_str_code(move))

    def encode_board(self):
        return np.asarray(self.board, dtype=np.int8).reshape(64).tobytes()

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
