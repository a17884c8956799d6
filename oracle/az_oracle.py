"""Test infrastructure: CPU restatement of the reference AlphaZero tree search for TicTacToe
(lzero/mcts/ctree/ctree_alphazero/mcts_alphazero.cpp:47-254, node_alphazero.h:9-80), one root at a
time, with the reference's number types: Node.prior_p / value_sum float32, visit_count int, the pUCT
score in double (parent.visit_count, no -1), first strict maximum over children in action order,
update_recursive with alternating signs (self_play_mode). Root noise: the reference's
default-seeded gamma vectors (oracle/az_noise.cpp, libstdc++). Pinned by tests/golden/az_*.npz.
"""
import ctypes
import math
import os

import numpy as np

from .tictactoe import SimTicTacToe

HERE = os.path.dirname(os.path.abspath(__file__))
_lib = None


def noise_table(alpha, max_n=9):
    global _lib
    if _lib is None:
        _lib = ctypes.CDLL(os.path.join(HERE, "liblzoracle_az.so"))
        _lib.lzo_az_noise_table.argtypes = [ctypes.c_double, ctypes.c_int, ctypes.c_void_p]
    out = np.zeros(max_n * max_n, np.float64)
    _lib.lzo_az_noise_table(float(alpha), int(max_n), out.ctypes.data)
    return out.reshape(max_n, max_n)


f32 = np.float32


class Node:
    __slots__ = ("parent", "prior", "visit", "value_sum", "children")

    def __init__(self, parent=None, prior=1.0):
        self.parent, self.prior = parent, f32(prior)
        self.visit, self.value_sum = 0, f32(0.0)
        self.children = {}

    def value(self):
        return f32(0.0) if self.visit == 0 else f32(self.value_sum / f32(self.visit))

    def update_recursive(self, v):
        node, v = self, f32(v)
        while node is not None:
            node.visit += 1
            node.value_sum = f32(node.value_sum + v)
            node, v = node.parent, f32(-v)


def ucb(parent, child, base, init):
    pb_c = math.log((parent.visit + base + 1) / base) + init
    pb_c *= math.sqrt(parent.visit) / (child.visit + 1)
    return pb_c * float(child.prior) + float(child.value())


def expand(node, env, pv):
    priors, value = pv(env.board.reshape(-1), env.legal_actions)
    legal = set(env.legal_actions)
    for a in sorted(priors):
        if a in legal:
            node.children[a] = Node(node, priors[a])
    return value


def search(board, start_player_index, sims, pv, sample, base=19652.0, init=1.25, alpha=0.3, frac=0.25, table=None,
           return_values=False):
    """Root visit counts [9] of MCTS.get_next_action (the action_probs it returns x sims at T=1);
    with return_values also the root children's value_sum float32 [9] and the root's (visit, value_sum)."""
    env = SimTicTacToe()
    root = Node()
    env.reset(start_player_index, board)
    expand(root, env, pv)
    if sample:
        tab = noise_table(alpha) if table is None else table
        acts = sorted(root.children)
        nz = tab[len(acts) - 1]
        for i, a in enumerate(acts):
            c = root.children[a]
            c.prior = f32(float(c.prior) * (1 - frac) + nz[i] * frac)
    for _ in range(sims):
        env.reset(start_player_index, board)
        node = root
        while node.children:
            best, action, child = -9999999.0, -1, None
            legal = set(env.legal_actions)
            for a in sorted(node.children):
                if a in legal:
                    s = ucb(node, node.children[a], base, init)
                    if s > best:
                        best, action, child = s, a, node.children[a]
            if child is None:
                break
            env.step(action)
            node = child
        done, winner = env.get_done_winner()
        if not done:
            leaf = expand(node, env, pv)
        else:
            leaf = 0.0 if winner == -1 else (1.0 if env.current_player == winner else -1.0)
        node.update_recursive(-leaf)
    visits = np.zeros(9, np.int64)
    vsums = np.zeros(9, np.float32)
    for a, c in root.children.items():
        visits[a] = c.visit
        vsums[a] = c.value_sum
    if return_values:
        return visits, vsums, (root.visit, root.value_sum)
    return visits
