"""List-in / list-out tree API with the exact surface of LightZero's Cython ctree modules.

Mirrors ``lzero/mcts/ctree/ctree_muzero/mz_tree.pyx:5-107`` (MuZero) and
``lzero/mcts/ctree/ctree_efficientzero/ez_tree.pyx:6-121`` (EfficientZero, ``is_reset``):
classes ``MinMaxStatsList``, ``ResultsWrapper``, ``Roots`` and the functions
``batch_traverse`` / ``batch_backpropagate``. Arguments typed ``list`` in the .pyx raise
``TypeError`` for anything else, as Cython does. The trees live on the GPU (lightzero_amd.tree);
each call stages its Python lists through HBM. The fast path that keeps everything on the
device is ``lightzero_amd.mcts_ctree`` (search loop) — this module is the compatibility
surface for code that drives the tree by hand.
"""
import numpy as np
import torch

from ..tree import POOL, new_minmax, next_seed, seed_tensor

_DEFAULT_SIMS = 64


def _require_list(name, v):
    if not isinstance(v, list):
        raise TypeError(f"Argument '{name}' has incorrect type (expected list, got {type(v).__name__})")


def _f32(v):
    return float(np.float32(v))


class MinMaxStatsList:
    """CMinMaxStatsList (common_lib/cminimax.cpp:47-66): one (max, min, delta) per root, in HBM."""

    def __init__(self, num):
        self.num = int(num)
        self._delta = 0.0
        self._buf = None

    def set_delta(self, value_delta_max):
        self._delta = _f32(value_delta_max)
        if self._buf is not None:
            self._buf[:, 2] = self._delta

    def _device(self, device):
        if self._buf is None or self._buf.device != device:
            self._buf = new_minmax(self.num, self._delta, device)
        return self._buf


class ResultsWrapper:
    """CSearchResults holder (mz_tree.pyx:18-25); the search paths themselves stay in the tree."""

    def __init__(self, num):
        self.num = int(num)
        self._search_lens = []

    def get_search_len(self):
        return list(self._search_lens)


class _RootsBase:
    EZ = False

    def __init__(self, root_num, legal_actions_list, fast_rng=False):
        self.fast_rng = bool(fast_rng)
        self.root_num = int(root_num)
        self._legal_list = [list(map(int, l)) for l in legal_actions_list]
        self._mask = None
        if len(self._legal_list) < self.root_num:
            raise IndexError("legal_actions_list shorter than root_num")
        self.tree = None
        self._sims = _DEFAULT_SIMS

    @classmethod
    def from_action_mask(cls, action_mask, fast_rng=False):
        """Roots whose legal lists come from an [N, A] {0, 1} action mask ON THE DEVICE (not in the
        reference; its callers build `[[i for i, x in enumerate(mask[j]) if x == 1] ...]` on the host,
        game_buffer_muzero.py:587-594): legal action j of root i = the j-th set bit of row i, computed
        by a stable sort on the device, no host copy. The host list view is built only if asked for."""
        m = action_mask.detach().to(torch.int32)
        N, A = m.shape
        r = cls.__new__(cls)
        r.fast_rng, r.root_num, r._legal_list, r._mask = bool(fast_rng), int(N), None, m
        r.tree, r._sims = None, _DEFAULT_SIMS
        count = m.sum(dim=1, dtype=torch.int32)
        order = torch.argsort(1 - m, dim=1, stable=True).to(torch.int32)  # set bits first, ascending
        cols = torch.arange(A, device=m.device, dtype=torch.int32).unsqueeze(0)
        legal = torch.where(cols < count.unsqueeze(1), order, torch.full_like(order, -1)).contiguous()
        r._legal_dev, r._legal_dev_key = (legal, count.contiguous()), (A, str(m.device))
        return r

    @property
    def legal_actions_list(self):
        if self._legal_list is None:  # (from_action_mask roots: the host view on demand)
            self._legal_list = [torch.nonzero(row).flatten().tolist() for row in self._mask.cpu()]
        return self._legal_list

    @property
    def num(self):
        return self.root_num

    def _acquire(self, A, device):
        if self.tree is not None and self.tree.A == A and self.tree.device == device:
            return self.tree
        if self.tree is not None:
            POOL.release(self.tree)
        self.tree = POOL.acquire(self.root_num, A, self._sims, self.EZ, self.fast_rng, device)
        return self.tree

    def _prepare(self, noise_weight, noises, rewards, logits, to_play, device=None):
        B = self.root_num
        logits = np.asarray(logits, dtype=np.float32).reshape(B, -1)
        A = logits.shape[1]
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        t = self._acquire(A, dev)
        legal = np.full((B, A), -1, np.int32)
        count = np.zeros(B, np.int32)
        nz = np.zeros((B, A), np.float32) if noises is not None else None
        for i in range(B):
            l = self.legal_actions_list[i]
            if len(l) > A or any(a < 0 or a >= A for a in l):
                raise ValueError(f"root {i}: legal actions {l} outside action space {A}")
            legal[i, :len(l)] = l
            count[i] = len(l)
            if nz is not None:
                row = np.asarray(noises[i], dtype=np.float32).reshape(-1)
                n = len(l) if len(l) > 0 else A
                if row.shape[0] < n:
                    raise IndexError(f"root {i}: {row.shape[0]} noises for {n} legal actions")
                nz[i, :n] = row[:n]
        g = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dtype=dt)).to(dev, non_blocking=False)
        t.prepare(g(legal, np.int32), g(count, np.int32), None if nz is None else g(nz, np.float32),
                  _f32(noise_weight), g(np.asarray(rewards, np.float32).reshape(B), np.float32), g(logits, np.float32),
                  g(np.asarray(to_play, np.int32).reshape(B), np.int32))

    def prepare(self, root_noise_weight, noises, value_prefix_pool, policy_logits_pool, to_play_batch):
        _require_list("noises", noises)
        _require_list("value_prefix_pool", value_prefix_pool)
        _require_list("policy_logits_pool", policy_logits_pool)
        self._prepare(root_noise_weight, noises, value_prefix_pool, policy_logits_pool, list(to_play_batch))

    def prepare_no_noise(self, value_prefix_pool, policy_logits_pool, to_play_batch):
        _require_list("value_prefix_pool", value_prefix_pool)
        _require_list("policy_logits_pool", policy_logits_pool)
        self._prepare(0.0, None, value_prefix_pool, policy_logits_pool, list(to_play_batch))

    def prepare_device(self, root_noise_weight, noises, rewards, logits, to_play):
        """Device-tensor variant (not in the reference): all arguments torch tensors on the GPU."""
        t, legal, count = self.device_legal(logits.shape[-1], logits.device)
        t.prepare(legal, count,
                  None if noises is None else noises.to(logits.device, torch.float32).contiguous(),
                  _f32(root_noise_weight), rewards.to(logits.device, torch.float32).contiguous(),
                  logits.to(logits.device, torch.float32).contiguous(), to_play.to(logits.device, torch.int32).contiguous())

    def device_legal(self, A, dev):
        """(tree, legal int32 [B, A], count int32 [B]) on `dev`: the device tree for A actions and the
        root legal lists uploaded once per Roots object (so preparation can be captured in a graph)."""
        B = self.root_num
        t = self._acquire(A, dev)
        key = (A, str(dev))
        if getattr(self, "_legal_dev_key", None) != key:
            # the legal lists are fixed per Roots object: upload once (no host copy on later calls,
            # so the call can be captured in a HIP graph)
            rows = self.legal_actions_list[:B]
            legal = np.full((B, A), -1, np.int32)
            count = np.zeros(B, np.int32)
            for i, l in enumerate(rows):
                legal[i, :len(l)] = l
                count[i] = len(l)
            self._legal_dev = (torch.from_numpy(legal).to(dev), torch.from_numpy(count).to(dev))
            self._legal_dev_key = key
        legal, count = self._legal_dev
        return t, legal, count

    def get_trajectories(self):
        if self.tree is None:
            return [[] for _ in range(self.root_num)]
        tr = self.tree.trajectories(self.tree.sims_capacity + 2).cpu().numpy()
        self.tree.check_once()
        return [[int(a) for a in row if a >= 0] for row in tr]

    def get_distributions(self):
        if self.tree is None:
            return [[] for _ in range(self.root_num)]
        d = self.tree.distributions().cpu().numpy()
        # once per search, by whichever getter runs first: a timed-out look-back
        # would leave a wrong tie-break stream; the words are cleared as they are read
        self.tree.check_once()
        return [[int(v) for v in row if v >= 0] for row in d]

    def get_values(self):
        if self.tree is None:
            return [0.0] * self.root_num
        v = self.tree.values().cpu().numpy()
        self.tree.check_once()
        return [float(x) for x in v]

    def clear(self):
        if self.tree is not None:
            POOL.release(self.tree)
            self.tree = None

    def __del__(self):
        try:
            self.clear()
        except Exception:
            pass


def _traverse(roots, pb_c_base, pb_c_init, discount_factor, min_max_stats_lst, results, virtual_to_play_batch,
              seed=None, reuse=None):
    if not isinstance(pb_c_base, (int, np.integer)):
        raise TypeError("an integer is required for pb_c_base")
    _require_list("virtual_to_play_batch", virtual_to_play_batch)
    t = roots.tree
    if t is None:
        raise RuntimeError("batch_traverse: roots not prepared")
    dev = t.device
    mm = min_max_stats_lst._device(dev)
    vtp = torch.tensor(np.asarray(virtual_to_play_batch, np.int32)[:t.B], device=dev)
    s = seed_tensor(next_seed() if seed is None else seed, dev)
    if reuse is None and getattr(t, "_reuse", None) is not None:
        t.set_reuse(None)
    if reuse is not None:
        t.set_reuse(*reuse)
    t.traverse(mm, s, vtp, int(pb_c_base), _f32(pb_c_init), _f32(discount_factor))
    out = torch.stack([t.x, t.y, t.action, t.vtp, t.search_len]).cpu().numpy()
    t.check_once()  # (already synchronised) this traverse's look-back / draw table intact
    results._search_lens = out[4].tolist()
    results._tree = t
    y = out[1]
    if reuse is not None:
        # latent_state_index_in_batch as the reference reports it: the parent's batch_index, i.e. its
        # position among the envs that ran inference in the parent's simulation (cnode.cpp:920)
        bidx = getattr(roots, "_batch_index", {})
        y = np.array([bidx[x][i] if x > 0 and x in bidx else i for i, x in enumerate(out[0])], np.int64)
    return out[0].tolist(), y.tolist(), out[2].tolist(), out[3].tolist()


def _backprop(current_latent_state_index, discount_factor, value_prefixs, values, policies, min_max_stats_lst,
              results, to_play_batch, is_reset_list=None):
    _require_list("value_prefixs", value_prefixs)
    _require_list("values", values)
    _require_list("policies", policies)
    _require_list("to_play_batch", to_play_batch)
    t = getattr(results, "_tree", None)
    if t is None:
        raise RuntimeError("batch_backpropagate: results do not come from batch_traverse")
    cur = int(current_latent_state_index)
    if 1 + t.A * (cur + 1) > 1 + t.A * (t.sims_capacity + 1):
        t.reserve(max(cur + 1, 2 * t.sims_capacity))
    dev = t.device
    B = t.B
    g = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dtype=dt)).to(dev)
    rs = None if is_reset_list is None else g(np.asarray(is_reset_list, np.int32).reshape(B), np.int32)
    t.backprop(cur, _f32(discount_factor), min_max_stats_lst._device(dev), g(np.asarray(value_prefixs).reshape(B), np.float32),
               g(np.asarray(values).reshape(B), np.float32), g(np.asarray(policies, np.float32).reshape(B, t.A), np.float32),
               g(np.asarray(to_play_batch, np.int32).reshape(B), np.int32), rs)


def _traverse_with_reuse(roots, pb_c_base, pb_c_init, discount_factor, min_max_stats_lst, results,
                         virtual_to_play_batch, true_action, reuse_value):
    """batch_traverse_with_reuse (mz_tree.pyx:102-107)."""
    _require_list("true_action", true_action)
    _require_list("reuse_value", reuse_value)
    t = roots.tree
    if t is None:
        raise RuntimeError("batch_traverse_with_reuse: roots not prepared")
    B = t.B
    ta = torch.from_numpy(np.asarray(true_action[:B], np.int32)).to(t.device)
    rv = torch.from_numpy(np.asarray(reuse_value[:B], np.float32)).to(t.device)
    x, y, a, vtp = _traverse(roots, pb_c_base, pb_c_init, discount_factor, min_max_stats_lst, results,
                             virtual_to_play_batch, reuse=(ta, rv))
    results._roots = roots
    return x, y, a, vtp


def _backprop_with_reuse(current_latent_state_index, discount_factor, value_prefixs, values, policies,
                         min_max_stats_lst, results, to_play_batch, no_inference_lst, reuse_lst, reuse_value_lst,
                         is_reset_list=None):
    """batch_backpropagate_with_reuse (mz_tree.pyx:84-93): the outputs arrive compacted to the envs
    that ran inference (every env not in no_inference_lst, in env order); they are scattered back
    to env rows, the device backup derives the no-inference / reuse cases from the tree itself
    (the same rule the caller used to build the two lists) and reads the reuse values."""
    for n, v in (("no_inference_lst", no_inference_lst), ("reuse_lst", reuse_lst),
                 ("reuse_value_lst", reuse_value_lst)):
        _require_list(n, v)
    t = getattr(results, "_tree", None)
    if t is None or getattr(t, "_reuse", None) is None:
        raise RuntimeError("batch_backpropagate_with_reuse: results do not come from batch_traverse_with_reuse")
    B, A = t.B, t.A
    skip = set(int(i) for i in no_inference_lst if int(i) >= 0)
    inf = [i for i in range(B) if i not in skip]
    if len(values) != len(inf) or len(value_prefixs) != len(inf) or len(policies) != len(inf):
        raise ValueError("batch_backpropagate_with_reuse: output lists must cover exactly the inferred envs")
    full_r = np.zeros(B, np.float32)
    full_v = np.zeros(B, np.float32)
    full_p = np.zeros((B, A), np.float32)
    if inf:
        full_r[inf] = np.asarray(value_prefixs, np.float32)
        full_v[inf] = np.asarray(values, np.float32)
        full_p[inf] = np.asarray(policies, np.float32).reshape(len(inf), A)
    rv = torch.from_numpy(np.asarray(reuse_value_lst[:B], np.float32)).to(t.device)
    t.set_reuse(t._reuse[0], rv)
    cur = int(current_latent_state_index)
    roots = getattr(results, "_roots", None)
    if roots is not None:
        if not hasattr(roots, "_batch_index"):
            roots._batch_index = {}
        roots._batch_index[cur] = {i: n for n, i in enumerate(inf)}
    if is_reset_list is not None and len(is_reset_list) != B:
        raise ValueError("batch_backpropagate_with_reuse: is_reset_list must hold one flag per env (len == batch): "
                         "the reference builds it over the inferred envs only and then reads it by env index "
                         "(ctree_efficientzero/lib/cnode.cpp:638), which is undefined once an env skips inference; "
                         "pass search_len % lstm_horizon_len == 0 for every env")
    _backprop(cur, discount_factor, full_r.tolist(), full_v.tolist(), full_p.tolist(), min_max_stats_lst, results,
              to_play_batch, is_reset_list)
    t.set_reuse(None)
