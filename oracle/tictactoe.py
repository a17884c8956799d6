"""Test infrastructure: TicTacToe simulate-env restated for driving the reference AlphaZero tree
(lzero/mcts/ctree/ctree_alphazero/mcts_alphazero.cpp) and the CPU restatement.

Restates the parts of zoo/board_games/tictactoe/envs/tictactoe_env.py the MCTS calls
(reset :131-170 with alphazero_mcts_ctree byte states, step / _player_step :209-224, :312-348 in
self_play_mode, legal_actions :102-104, get_done_winner via get_done_winner_cython.pyx, current_state
:350-376, current_player / next_player :489-504). The real env imports DI-engine (not installed).
"""
import numpy as np


def done_winner(board):
    """get_done_winner_cython.pyx: (done, winner) with winner 1/2, or -1 for draw / not over."""
    b = np.asarray(board, dtype=np.int32).reshape(3, 3)
    has_legal = False
    dirs = ((1, -1), (1, 0), (1, 1), (0, 1))
    for i in range(3):
        for j in range(3):
            if b[i, j] == 0:
                has_legal = True
                continue
            player = b[i, j]
            start = 0 if j > 0 else 1
            end = 4 if j < 2 else 3
            for d in dirs[start:end]:
                x, y, count = i, j, 0
                for _ in range(3):
                    if x < 0 or x >= 3 or y < 0 or y >= 3 or b[x, y] != player:
                        break
                    x += d[0]
                    y += d[1]
                    count += 1
                    if count == 3:
                        return True, int(player)
    return (not has_legal), -1


class _Space:
    n = 9


class SimTicTacToe:
    def __init__(self, scale=True):
        self.scale = scale
        self.battle_mode = 'self_play_mode'
        self.battle_mode_in_simulation_env = 'self_play_mode'
        self.action_space = _Space()
        self.players = [1, 2]
        self.board = np.zeros((3, 3), np.int32)
        self._current_player = 1

    def reset(self, start_player_index=0, init_state=None, katago_policy_init=False, katago_game_state=None):
        self._current_player = self.players[start_player_index]
        if init_state is not None:
            if isinstance(init_state, (bytes, bytearray)):
                init_state = np.frombuffer(init_state, dtype=np.int32)
            self.board = np.array(init_state, dtype=np.int32).reshape(3, 3)
        else:
            self.board = np.zeros((3, 3), np.int32)

    @property
    def legal_actions(self):
        return [i * 3 + j for i in range(3) for j in range(3) if self.board[i, j] == 0]

    @property
    def current_player(self):
        return self._current_player

    @property
    def next_player(self):
        return 2 if self._current_player == 1 else 1

    def get_done_winner(self):
        return done_winner(self.board)

    def step(self, action):
        row, col = action // 3, action % 3
        assert self.board[row, col] == 0, "illegal action in simulation"
        self.board[row, col] = self._current_player
        self._current_player = self.next_player

    def current_state(self):
        cur = np.where(self.board == self.current_player, 1, 0)
        opp = np.where(self.board == self.next_player, 1, 0)
        tp = np.full((3, 3), self.current_player)
        raw = np.array([cur, opp, tp], dtype=np.float32)
        return raw, (raw / 2 if self.scale else raw)


def board_code(board):
    """base-3 code of the absolute board (cell k weight 3^k)"""
    b = np.asarray(board, dtype=np.int64).reshape(-1)
    return int(sum(int(b[k]) * 3 ** k for k in range(9)))


def scripted_policy_value(board, legal):
    """Deterministic float-exact network stand-in: priors (1 + (7h + 13a) % 16) / 64 over the legal
    actions, value ((31h) % 129 - 64) / 64 (h = board_code)."""
    h = board_code(board)
    priors = {int(a): (1 + (7 * h + 13 * int(a)) % 16) / 64.0 for a in legal}
    value = ((31 * h) % 129 - 64) / 64.0
    return priors, value


def random_boards(n, seed, max_moves=4):
    """n positions reached by k ~ U{0..max_moves} random legal moves from empty (player 1 first),
    not terminal; returns (boards int32 [n][9], start_player_index [n])."""
    rng = np.random.default_rng(seed)
    boards, starts = [], []
    while len(boards) < n:
        b = np.zeros(9, np.int32)
        p = 1
        for _ in range(int(rng.integers(0, max_moves + 1))):
            legal = np.nonzero(b == 0)[0]
            b[rng.choice(legal)] = p
            p = 2 if p == 1 else 1
            if done_winner(b)[0]:
                break
        if done_winner(b)[0]:
            continue
        boards.append(b)
        starts.append(0 if p == 1 else 1)
    return np.stack(boards), np.array(starts, np.int32)
