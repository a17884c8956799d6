"""CPU restatement of LightZero's pure-Python MuZero tree (config 1's CPU baseline).

TEST / BASELINE INFRASTRUCTURE ONLY: imported by tests/ (parity against the reference's own ptree,
tests/golden/ptree_*.npz) and by tools/ptree_bench.py (the config-1 CPU timing). Nothing in
lightzero_amd/ imports it.

Restates /root/reference/lzero/mcts/ptree/ptree_mz.py and minimax.py, and the search loop of
lzero/mcts/tree_search/mcts_ptree.py:92-194, keeping the reference's execution model on purpose — one
Python object per node, children in a dict, a torch.softmax per expansion, float64 Python arithmetic,
Python's `random.choice` for ties — because this is what config 1 times. Semantics (all differ from
the ctree, hence no parity with the GPU search): the pUCT parent count is the parent's
visit_count (no -1), min-max starts at (+1e6, -inf) and value_delta_max stays 0 (set_delta is never
called), and batch_traverse's parent_q is initialised once per call, so a walk's first non-root level
starts from the previous root's last mean_q.
"""
import math

import numpy as np
import torch

FLOAT_MAX = 1000000.0  # minimax.py:4-5
FLOAT_MIN = -float("inf")


class MinMax:
    """MinMaxStats (minimax.py:8-76): delta 0 unless set."""
    __slots__ = ("maximum", "minimum", "delta")

    def __init__(self):
        self.minimum, self.maximum, self.delta = FLOAT_MAX, FLOAT_MIN, 0

    def update(self, v):
        if v > self.maximum:
            self.maximum = v
        if v < self.minimum:
            self.minimum = v

    def normalize(self, v):
        d = self.maximum - self.minimum
        if d > 0:
            return (v - self.minimum) / (self.delta if d < self.delta else d)
        return v


class PNode:
    """Node (ptree_mz.py:14-186)."""
    __slots__ = ("prior", "legal", "visit_count", "value_sum", "best_action", "to_play", "reward", "children",
                 "simulation_index", "batch_index")

    def __init__(self, prior, legal=None):
        self.prior, self.legal = prior, legal
        self.visit_count, self.value_sum, self.best_action, self.to_play, self.reward = 0, 0, -1, -1, 0
        self.children = {}
        self.simulation_index = self.batch_index = 0

    def expand(self, to_play, sim, b, reward, logits):  # ptree_mz.py:46-69 (float32 torch softmax)
        self.to_play = to_play
        if self.legal is None:
            self.legal = np.arange(len(logits))
        self.simulation_index, self.batch_index, self.reward = sim, b, reward
        priors = torch.softmax(torch.tensor([logits[a] for a in self.legal]), dim=0).tolist()
        for j, a in enumerate(self.legal):
            self.children[int(a)] = PNode(priors[j])

    @property
    def value(self):  # ptree_mz.py:175-186
        return 0 if self.visit_count == 0 else self.value_sum / self.visit_count

    def mean_q(self, is_root, parent_q, disc):  # ptree_mz.py:88-115
        tq, tv = 0.0, 0
        for a in self.legal:
            c = self.children[int(a)]
            if c.visit_count > 0:
                tq += c.reward + disc * c.value
                tv += 1
        return tq / tv if (is_root and tv > 0) else (parent_q + tq) / (tv + 1)


class PRoots:
    """Roots (ptree_mz.py:189-303)."""

    def __init__(self, n, legal_actions_list):
        self.num = n
        self.roots = [PNode(0, legal_actions_list[i]) if isinstance(legal_actions_list, list)
                      else PNode(0, np.arange(legal_actions_list)) for i in range(n)]

    def prepare(self, noise_weight, noises, rewards, policies, to_play):  # :217-242
        for i, r in enumerate(self.roots):
            r.expand(-1 if to_play is None else to_play[i], 0, i, rewards[i], policies[i])
            for j, a in enumerate(r.legal):
                c = r.children[int(a)]
                c.prior = c.prior * (1 - noise_weight) + noises[i][j] * noise_weight
            r.visit_count += 1

    def prepare_no_noise(self, rewards, policies, to_play):  # :244-259
        for i, r in enumerate(self.roots):
            r.expand(-1 if to_play is None else to_play[i], 0, i, rewards[i], policies[i])
            r.visit_count += 1

    def get_distributions(self):  # :280-291 via get_children_distribution :133-150
        return [[r.children[int(a)].visit_count for a in r.legal] if r.children else [0 for _ in r.legal]
                for r in self.roots]

    def get_values(self):
        return [r.value for r in self.roots]

    def get_trajectories(self):  # :117-131
        out = []
        for r in self.roots:
            t, n = [], r
            while n.best_action >= 0:
                t.append(n.best_action)
                n = n.children[int(n.best_action)]
            out.append(t)
        return out


def ucb(c, mm, parent_mean_q, parent_visits, pb_c_base, pb_c_init, disc, players):  # ptree_mz.py:370-419
    pb_c = (math.log((parent_visits + pb_c_base + 1) / pb_c_base) + pb_c_init) * (math.sqrt(parent_visits) / (c.visit_count + 1))
    if c.visit_count == 0:
        v = parent_mean_q
    else:
        v = c.reward + disc * (c.value if players == 1 else -c.value)
    v = mm.normalize(v)
    v = 0 if v < 0 else (1 if v > 1 else v)
    return pb_c * c.prior + v


def select_child(node, mm, pb_c_base, pb_c_init, disc, mean_q, players, rng):  # ptree_mz.py:330-367
    best, ties = -np.inf, []
    for a in node.legal:
        s = ucb(node.children[int(a)], mm, mean_q, node.visit_count, pb_c_base, pb_c_init, disc, players)
        if best < s:
            best = s
            ties = [a]
        elif s >= best - 0.000001:
            ties.append(a)
    return rng.choice(ties) if ties else 0


class PResults:
    __slots__ = ("num", "paths", "nodes", "x", "y", "actions", "lens")

    def __init__(self, num):
        self.num = num


def batch_traverse(roots, pb_c_base, pb_c_init, disc, mms, res, vtp, rng):  # ptree_mz.py:422-508
    B = res.num
    res.lens, res.actions, res.nodes, res.x, res.y = [None] * B, [None] * B, [None] * B, [None] * B, [None] * B
    v0 = vtp if not isinstance(vtp, (list, tuple, np.ndarray)) else vtp[0]
    players = 2 if v0 in (1, 2) else 1
    res.paths = [[] for _ in range(B)]
    parent_q = 0.0  # once per call (the reference's scope)
    for i in range(B):
        node, is_root, slen = roots.roots[i], 1, 0
        path = res.paths[i]
        path.append(node)
        while node.children:
            mean_q = node.mean_q(is_root, parent_q, disc)
            is_root, parent_q = 0, mean_q
            a = select_child(node, mms[i], pb_c_base, pb_c_init, disc, mean_q, players, rng)
            if players == 2:
                vtp[i] = 2 if vtp[i] == 1 else 1
            node.best_action = a
            node = node.children[int(a)]
            path.append(node)
            slen += 1
            parent = path[-2]
            res.x[i], res.y[i], res.actions[i], res.lens[i], res.nodes[i] = (parent.simulation_index, parent.batch_index,
                                                                              a, slen, node)
    return res.x, res.y, res.actions, vtp


def backpropagate(path, mm, to_play, value, disc):  # ptree_mz.py:511-562
    b = value
    if to_play is None or to_play == -1:
        for node in reversed(path):
            node.value_sum += b
            node.visit_count += 1
            mm.update(node.reward + disc * node.value)
            b = node.reward + disc * b
    else:
        for node in reversed(path):
            node.value_sum += b if node.to_play == to_play else -b
            node.visit_count += 1
            mm.update(node.reward + disc * -node.value)
            b = (-node.reward if node.to_play == to_play else node.reward) + disc * b


def batch_backpropagate(sim, disc, rewards, values, policies, mms, res, to_play):  # ptree_mz.py:565-602
    for i in range(res.num):
        tp = -1 if to_play is None else to_play[i]
        res.nodes[i].expand(tp, sim, i, rewards[i], policies[i])
        backpropagate(res.paths[i], mms[i], 0 if to_play is None else to_play[i], values[i], disc)


def search(roots, recurrent, latent_roots, to_play, S, pb_c_base=19652, pb_c_init=1.25, disc=0.997, rng=None,
           record=None):
    """MuZeroMCTSPtree.search (mcts_ptree.py:92-194) with `recurrent(latents, actions, k)` returning decoded
    (next_latents, rewards, values, policy_logits) as Python / numpy values; `rng` provides choice().
    record: optional dict receiving per-simulation x / y / action / search_len lists."""
    import random as _random
    rng = rng or _random
    B = roots.num
    pool = [latent_roots]
    mms = [MinMax() for _ in range(B)]
    for k in range(S):
        res = PResults(B)
        x, y, acts, vtp = batch_traverse(roots, pb_c_base, pb_c_init, disc, mms, res, to_play, rng)
        if record is not None:
            for key, v in (("x", x), ("y", y), ("action", acts), ("search_len", res.lens)):
                record.setdefault(key, []).append(list(v))
        lat = [pool[ix][iy] for ix, iy in zip(x, y)]
        nxt, rewards, values, logits = recurrent(lat, acts, k)
        pool.append(nxt)
        batch_backpropagate(k + 1, disc, rewards, values, logits, mms, res, vtp)
    return roots
