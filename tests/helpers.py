"""Shared test helpers: scripted networks, the host restatement of the search loop, and an
adapter that drives the GPU tree through the C ABI with the oracle's interface."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

from oracle.oracle import OracleTree  # noqa: E402  (test infrastructure)

PB_C_BASE, PB_C_INIT, DISC, VDM, NOISE_W = 19652, np.float32(1.25), np.float32(0.997), np.float32(0.01), np.float32(0.25)


def h_inverse_np(x):
    """h^-1 in float32, operation for operation as the device kernel (lzm_kernels.hip h_inverse)."""
    x = np.asarray(x, np.float32)
    a = np.abs(x)
    inner = np.float32(1.0) + np.float32(0.004) * ((a + np.float32(1.0)) + np.float32(0.001))
    tmp = (np.sqrt(inner).astype(np.float32) - np.float32(1.0)) * np.float32(np.float32(1.0) / np.float32(0.002))
    return (np.sign(x).astype(np.float32) * (tmp * tmp - np.float32(1.0))).astype(np.float32)


class ScriptedTables:
    """Deterministic per-(simulation, root) network outputs. Latents stay small integers, so
    every float op below is exact or a single IEEE rounding identical on host and device."""

    def __init__(self, B, S, A, seed, H=8, players=1, quant=False):
        rng = np.random.default_rng(seed)
        self.B, self.S, self.A, self.H = B, S, A, H
        if quant:
            self.r = rng.integers(-1, 2, size=(S, B)).astype(np.float32)
            self.v = rng.integers(-2, 3, size=(S, B)).astype(np.float32)
            self.p = rng.integers(0, 2, size=(S, B, A)).astype(np.float32)
        else:
            self.r = rng.normal(0, 0.5, size=(S, B)).astype(np.float32)
            self.v = rng.normal(0, 2.0, size=(S, B)).astype(np.float32)
            self.p = rng.normal(0, 1.0, size=(S, B, A)).astype(np.float32)
        self.lat0 = rng.integers(-3, 4, size=(B, H)).astype(np.float32)
        self.root_logits = rng.normal(0, 1, size=(B, A)).astype(np.float32)
        self.noises = rng.dirichlet([0.3] * A, size=B).astype(np.float32)
        if players == 1:
            self.to_play = np.full(B, -1, np.int32)
        else:
            self.to_play = rng.integers(1, 3, size=B).astype(np.int32)

    def step_np(self, k, lat, action):
        s = lat.sum(axis=1, dtype=np.float32)
        r = self.r[k] + np.float32(0.01) * s
        v = self.v[k] + np.float32(0.01) * s
        p = self.p[k] + np.float32(0.01) * lat[:, :1]
        nxt = lat + (action.astype(np.float32) + np.float32(1.0))[:, None]
        return nxt.astype(np.float32), r.astype(np.float32), v.astype(np.float32), p.astype(np.float32)


def make_scripted_model(tab, device):
    """torch module with the MuZero recurrent_inference surface over ScriptedTables (scalar heads)."""
    import torch

    class Out:
        pass

    class ScriptedModel(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.k = 0
            self.r = torch.from_numpy(tab.r).to(device)
            self.v = torch.from_numpy(tab.v).to(device)
            self.p = torch.from_numpy(tab.p).to(device)

        def recurrent_inference(self, latent, action):
            k = self.k
            self.k += 1
            s = latent.sum(dim=1)
            o = Out()
            o.reward = (self.r[k] + 0.01 * s).unsqueeze(1)
            o.value = (self.v[k] + 0.01 * s).unsqueeze(1)
            o.policy_logits = self.p[k] + 0.01 * latent[:, :1]
            o.latent_state = latent + (action.to(torch.float32) + 1.0).unsqueeze(1)
            return o

    return ScriptedModel()


def run_scripted_search_oracle(B, S, A, seed, players=1, quant=False, fast_rng=False):
    """Host restatement of MuZeroMCTSCtree.search (mcts_ctree.py:228-321) with the oracle tree."""
    tab = ScriptedTables(B, S, A, seed, players=players, quant=quant)
    t = OracleTree(B, A, S, fast_rng=fast_rng)
    legal = np.tile(np.arange(A, dtype=np.int32), (B, 1))
    t.set_legal(legal, np.full(B, A, np.int32))
    t.set_delta(VDM)
    t.prepare(NOISE_W, tab.noises, np.zeros(B, np.float32), tab.root_logits, tab.to_play)
    pool = [tab.lat0]
    rec = {k: np.zeros((S, B), np.int32) for k in ("x", "a", "len", "vtp")}
    for k in range(S):
        sd = (1000003 * seed + k) % 1000000
        x, y, a, vtp, slen = t.traverse(PB_C_BASE, PB_C_INIT, DISC, sd, tab.to_play)
        rec["x"][k], rec["a"][k], rec["len"][k], rec["vtp"][k] = x, a, slen, vtp
        lat = np.stack([pool[x[i]][i] for i in range(B)])
        nxt, r, v, p = tab.step_np(k, lat, a)
        t.backprop(k + 1, DISC, h_inverse_np(r), h_inverse_np(v), p, vtp)
        pool.append(nxt)
    rec.update(dist=t.distributions(), values=t.values(), traj=t.trajectories(S + 2))
    return rec


def run_scripted_search_gpu(B, S, A, seed, players=1, quant=False, fast_rng=False):
    """The drop-in MuZeroMCTSCtree.search on cuda:0 with the same scripted network."""
    import torch
    from lightzero_amd.mcts_ctree import MuZeroMCTSCtree
    from lightzero_amd.tree import SequentialSeeds, set_seed_source
    from lightzero_amd.utils import EasyDict

    tab = ScriptedTables(B, S, A, seed, players=players, quant=quant)
    dev = torch.device("cuda", 0)
    cfg = EasyDict(dict(num_simulations=S, discount_factor=float(DISC), device=dev,
                        model=dict(support_scale=300, categorical_distribution=False)))
    cls = MuZeroMCTSCtree
    old_mode = cls.rng_mode
    cls.rng_mode = "philox" if fast_rng else "glibc"
    try:
        mcts = cls(cfg)
        mcts.record = True
        roots = cls.roots(B, [list(range(A)) for _ in range(B)])
        roots.prepare(float(NOISE_W), [row.tolist() for row in tab.noises], [0.0] * B, tab.root_logits.tolist(),
                      tab.to_play.tolist())
        set_seed_source(SequentialSeeds(seed))
        try:
            mcts.search(roots, make_scripted_model(tab, dev), tab.lat0, tab.to_play.tolist())
        finally:
            set_seed_source(None)
        rec = mcts.last_record.numpy()
        out = dict(x=rec["x"], a=rec["action"], len=rec["search_len"], vtp=rec["vtp"])
        t = roots.tree
        out.update(dist=t.distributions().cpu().numpy(), values=t.values().cpu().numpy(),
                   traj=t.trajectories(S + 2).cpu().numpy())
        roots.clear()
        return out
    finally:
        cls.rng_mode = old_mode


class GpuTree:
    """OracleTree-shaped adapter over lightzero_amd.tree.DeviceTree (every call goes through
    the C ABI of liblzmcts.so), so oracle.replay_transcript can drive the GPU tree."""

    def __init__(self, num_roots, action_space, max_sims, ez=False, fast_rng=False):
        import torch
        from lightzero_amd.tree import DeviceTree
        self.torch = torch
        self.dev = torch.device("cuda", 0)
        self.t = DeviceTree(num_roots, action_space, max_sims, ez=ez, fast_rng=fast_rng, device=self.dev)
        self.B, self.A = num_roots, action_space
        self.legal = self.count = None
        self.delta = np.float32(0)
        self.mm = None

    def _d(self, a, dt):
        return self.torch.from_numpy(np.ascontiguousarray(a, dtype=dt)).to(self.dev)

    def set_legal(self, legal, count):
        self.legal, self.count = self._d(legal, np.int32), self._d(count, np.int32)

    def set_delta(self, d):
        self.delta = np.float32(d)

    def prepare(self, noise_weight, noises, rewards, logits, to_play):
        from lightzero_amd.tree import new_minmax
        if self.legal is None:
            self.set_legal(np.tile(np.arange(self.A, dtype=np.int32), (self.B, 1)), np.full(self.B, self.A, np.int32))
        self.t.prepare(self.legal, self.count, None if noises is None else self._d(noises, np.float32),
                       float(noise_weight), self._d(rewards, np.float32), self._d(logits, np.float32),
                       self._d(to_play, np.int32))
        self.mm = new_minmax(self.B, float(self.delta), self.dev)

    def traverse(self, pb_c_base, pb_c_init, discount, seed, vtp):
        from lightzero_amd.tree import seed_tensor
        self.t.traverse(self.mm, seed_tensor(seed, self.dev), self._d(vtp, np.int32), int(pb_c_base),
                        float(pb_c_init), float(discount))
        t = self.t
        out = self.torch.stack([t.x, t.y, t.action, t.vtp, t.search_len]).cpu().numpy()
        return tuple(out[i] for i in range(5))

    def backprop(self, cur, discount, rewards, values, logits, to_play, is_reset=None):
        self.t.backprop(cur, float(discount), self.mm, self._d(rewards, np.float32), self._d(values, np.float32),
                        self._d(logits, np.float32), self._d(to_play, np.int32),
                        None if is_reset is None else self._d(is_reset, np.int32))

    def distributions(self):
        return self.t.distributions().cpu().numpy()

    def values(self):
        return self.t.values().cpu().numpy()

    def trajectories(self, tmax=64):
        return self.t.trajectories(tmax).cpu().numpy()


def random_transcript(B, S, A, seed, players=1, ez=False, net="rand", ragged=False, noise=True):
    """A transcript-shaped dict whose responses are scripted (requests/outputs to be filled by
    the oracle) — used to compare GPU and oracle at sizes beyond the committed fixtures."""
    rng = np.random.default_rng(seed)
    legal_mask = np.ones((B, A), np.int8)
    if ragged:
        for i in range(B):
            k = int(rng.integers(1, A + 1))
            legal_mask[i] = 0
            legal_mask[i, rng.choice(A, size=k, replace=False)] = 1

    def tab(shape):
        if net == "zero":
            return np.zeros(shape, np.float32)
        if net == "quant":
            return rng.integers(-1, 2, size=shape).astype(np.float32)
        return rng.normal(0, 1, size=shape).astype(np.float32)

    noises = np.zeros((B, A), np.float32)
    for i in range(B):
        n = int(legal_mask[i].sum())
        noises[i, :n] = rng.dirichlet([0.3] * n)
    to_play = np.full(B, -1, np.int32) if players == 1 else rng.integers(1, 3, size=B).astype(np.int32)
    tr = dict(meta=np.array([B, S, A, players, int(noise), int(ez), 5]),
              consts=np.array([PB_C_BASE, 1.25, 0.997, 0.01, 0.25]),
              legal_mask=legal_mask, to_play=to_play, noises=noises, root_logits=tab((B, A)),
              root_reward=np.zeros(B, np.float32) if not ez else tab((B,)),
              seeds=np.array([(1000003 * seed + k) % 1000000 for k in range(S)]),
              resp_reward=tab((S, B)) * np.float32(0.5), resp_value=tab((S, B)), resp_logits=tab((S, B, A)),
              resp_is_reset=np.zeros((S, B), np.int32))
    return tr


def run_transcript(tr, factory, fast_rng=False):
    """Drive a tree (oracle or GPU) over a transcript's inputs; return every request and output."""
    from oracle.oracle import legal_from_mask
    B, S, A, players, noise, ez, horizon = [int(v) for v in tr["meta"]]
    t = factory(B, A, S, ez=bool(ez), fast_rng=fast_rng)
    legal, cnt = legal_from_mask(tr["legal_mask"])
    t.set_legal(legal, cnt)
    t.set_delta(VDM)
    t.prepare(NOISE_W, tr["noises"] if noise else None, tr["root_reward"], tr["root_logits"], tr["to_play"])
    rec = {k: np.zeros((S, B), np.int32) for k in ("x", "y", "a", "vtp", "len")}
    for k in range(S):
        out = t.traverse(PB_C_BASE, PB_C_INIT, DISC, int(tr["seeds"][k]), tr["to_play"])
        for name, v in zip(("x", "y", "a", "vtp", "len"), out):
            rec[name][k] = v
        is_reset = (out[4] % horizon == 0).astype(np.int32) if ez else None
        t.backprop(k + 1, DISC, tr["resp_reward"][k], tr["resp_value"][k], tr["resp_logits"][k], out[3], is_reset)
    rec.update(dist=t.distributions(), values=t.values(), traj=t.trajectories(S + 2))
    return rec


def az_scripted_pv_torch(state):
    """oracle.tictactoe.scripted_policy_value on the device, batched: the absolute board is rebuilt from
    the network input (current_state / 2: own stones, opponent stones, player-to-move plane)."""
    import torch
    player = torch.round(state[:, 2, 0, 0] * 2).to(torch.int64)  # 1 / 2
    cur = (state[:, 0] > 0).reshape(-1, 9).to(torch.int64)
    opp = (state[:, 1] > 0).reshape(-1, 9).to(torch.int64)
    board = cur * player[:, None] + opp * (3 - player)[:, None]
    pw = torch.pow(3, torch.arange(9, dtype=torch.int64, device=state.device))  # no host copy: graph-capturable
    h = (board * pw).sum(dim=1)
    a = torch.arange(9, dtype=torch.int64, device=state.device)
    priors = (1 + (7 * h[:, None] + 13 * a[None, :]) % 16).to(torch.float32) / 64.0
    value = ((31 * h) % 129 - 64).to(torch.float32) / 64.0
    return priors, value


def tie_list(scores):
    """cselect_child's order-dependent tie list (cnode.cpp:551-596) over one level's scores, in float32:
    scan in action order from max_score = FLOAT_MIN (-1e6); a score above the max restarts the list,
    one within 1e-6 below it joins (non-legal actions carry -inf and never join)."""
    mx = np.float32(-1e6)
    eps = np.float32(1e-6)
    lst = []
    for a, s in enumerate(np.asarray(scores, np.float32)):
        if not np.isfinite(s):
            continue
        if mx < s:
            mx = s
            lst = [a]
        elif s >= np.float32(mx - eps):
            lst.append(a)
    return lst
