"""Drop-in ``MuZeroMCTSCtree`` / ``EfficientZeroMCTSCtree`` with the search loop on the GPU.

Same class surface as /root/reference/lzero/mcts/tree_search/mcts_ctree.py:172-420 (MuZero) and
:623-827 (EfficientZero): class attribute ``config``, ``default_config()``, ``__init__(cfg)``,
classmethod ``roots(n, legal_actions)`` and ``search(...)``. The difference is where the
per-simulation loop (mcts_ctree.py:255-321) runs: here every step is a device kernel or a
device-resident model call on one stream —

    traverse (select, HIP)  ->  gather leaf latents (HIP)  ->  model.recurrent_inference
    ->  decode value/reward supports + expand + backup (one HIP kernel, also files the new
        latents into the [S+1, B, ...] pool in HBM)

with no host round trip inside a search. The tree and the tie-break RNG follow the reference
bit for bit in the default parity mode (glibc rand() stream seeded per traverse, exactly one
draw per tree level), see lzm_kernels.hip.
"""
import copy
import os
import weakref
from collections import OrderedDict
from typing import Any, List, Union

import numpy as np
import torch

from . import _lib
from .ctree import ez_tree, mz_tree
from .conv_infer import FoldedCache
from .fused import NotPackable, PackedCache
from .scaling_transform import InverseScalarTransform
from .tree import DeviceTree, new_minmax, next_seed
from .utils import EasyDict


def _seeds(n, device):
    s = np.array([next_seed() for _ in range(n)], dtype=np.uint32).view(np.int32)
    return torch.from_numpy(s).to(device)


def _to_play_tensor(to_play_batch, B, device):
    if isinstance(to_play_batch, torch.Tensor):
        return to_play_batch.to(device=device, dtype=torch.int32).reshape(B)
    if isinstance(to_play_batch, (int, np.integer)):
        return torch.full((B,), int(to_play_batch), dtype=torch.int32, device=device)
    return torch.as_tensor(np.asarray(to_play_batch, dtype=np.int32).reshape(B), device=device)


def _usable_i32(x, n, device):
    """a contiguous int32 device tensor of n elements on `device` (readable by a kernel as is)"""
    return (isinstance(x, torch.Tensor) and x.dtype == torch.int32 and x.is_contiguous() and x.numel() == n
            and x.device == torch.device(device))


def _latent_tensor(x, device):
    if isinstance(x, torch.Tensor):
        return x.to(device=device, dtype=torch.float32)
    if isinstance(x, (list, tuple)):
        x = np.asarray(x)
    return torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32)).to(device)


class _Recorder:
    """Optional per-simulation record of what the tree requested and consumed (tests, tracing)."""

    def __init__(self, S, B, A, device):
        i32 = dict(dtype=torch.int32, device=device)
        self.x = torch.zeros((S, B), **i32)
        self.action = torch.zeros((S, B), **i32)
        self.search_len = torch.zeros((S, B), **i32)
        self.vtp = torch.zeros((S, B), **i32)
        self.decoded = torch.zeros((S, B, 2), dtype=torch.float32, device=device)
        self.policy_logits = torch.zeros((S, B, A), dtype=torch.float32, device=device)
        self.seeds = None

    def step(self, k, t, policy_logits):
        self.x[k].copy_(t.x)
        self.action[k].copy_(t.action)
        self.search_len[k].copy_(t.search_len)
        self.vtp[k].copy_(t.vtp)
        self.policy_logits[k].copy_(policy_logits)

    def numpy(self):
        return {k: getattr(self, k).cpu().numpy() for k in
                ("x", "action", "search_len", "vtp", "decoded", "policy_logits")} | {"seeds": self.seeds}


class _SearchBuffers:
    """Per (B, S, latent shape) device buffers reused across searches."""

    def __init__(self):
        self.key = None

    def get(self, B, S, shape, device, extra=()):
        key = (B, S, tuple(shape), str(device), tuple(extra))
        if key != self.key:
            self.pool = torch.empty((S + 1, B) + tuple(shape), dtype=torch.float32, device=device)
            self.net_in = torch.empty((B,) + tuple(shape), dtype=torch.float32, device=device)
            self.extra = [torch.empty((S + 1, B, e), dtype=torch.float32, device=device) for e in extra]
            self.extra_in = [torch.empty((B, e), dtype=torch.float32, device=device) for e in extra]
            self.mm = torch.empty((B, 4), dtype=torch.float32, device=device)
            self.vtp_in = torch.empty(B, dtype=torch.int32, device=device)
            self.seeds = torch.empty(S, dtype=torch.int32, device=device)
            self.key = key
        return self


_CUS = {}


def _device_cus(device):
    """compute units of `device` (the one-launch conv search needs one co-resident workgroup per root)"""
    key = str(device)
    if key not in _CUS:
        _CUS[key] = torch.cuda.get_device_properties(device).multi_processor_count
    return _CUS[key]


def _step_net(mcts, model):
    """the BN-folded recurrent step for the conv MuZeroModel / EfficientZeroModel family
    (conv_infer.FoldedConvNet, cfg.fold_network, default on), else the model itself"""
    if mcts._cfg.get('fold_network', True):
        net = mcts._folded.get(model)
        if net is not None:
            return net
    return model


class _GraphEntry:
    """One captured search: the graph together with everything its kernels point at — the
    buffers the inputs are copied into, the (folded) network whose weights it reads — so none of
    them can be freed or rebuilt while the graph may replay."""

    def __init__(self, graph, buf, net, model, tree):
        self.graph, self.buf, self.net = graph, buf, net
        self.model_ref, self.tree_ref = weakref.ref(model), weakref.ref(tree)

    def valid_for(self, model, tree):
        return self.model_ref() is model and self.tree_ref() is tree and tree.h is not None

    def replay(self):
        if self.net is not None and hasattr(self.net, "refresh"):
            self.net.refresh()  # re-fold in place if the parameters changed since capture
        self.graph.replay()


class _GraphCache:
    """LRU of captured searches keyed by (tree uid, tree generation, model, B, S, latent shape);
    entries whose tree or model died are dropped on lookup, the oldest beyond `cap` evicted."""

    def __init__(self, cap=4):
        self.cap = int(cap)
        self._d = OrderedDict()

    def __len__(self):
        return len(self._d)

    def get(self, key, model, tree):
        e = self._d.get(key)
        if e is None:
            return None
        if not e.valid_for(model, tree):
            del self._d[key]
            return None
        self._d.move_to_end(key)
        return e

    def put(self, key, entry):
        self._d[key] = entry
        self._d.move_to_end(key)
        for k in [k for k, e in self._d.items() if e.tree_ref() is None or e.model_ref() is None]:
            del self._d[k]
        while len(self._d) > self.cap:
            self._d.popitem(last=False)


def _graph_key(t, model, B, S, shape, extra=()):
    return (t.uid, t.generation, id(model), B, S, tuple(shape), tuple(extra))


def _fuse_traverse(cfg, t):
    """fold each simulation's traverse into the previous simulation's decode launch (parity mode with
    the look-back traverse; cfg.fuse_traverse, default off: measured even with the two launches at
    the conv configs; LZM_FUSE=0 forces it off)"""
    return (cfg.get('fuse_traverse', False) and not t.fast_rng and os.environ.get("LZM_FUSE", "1") != "0"
            and os.environ.get("LZM_TRAVERSE", "") != "serial")


class _HeadVerdicts:
    """The native conv step's head kernel writes ensure_softmax's verdict words for the tree's
    decode (one launch fewer per simulation); set for the duration of a loop."""

    def __init__(self, t, net, buf, on):
        self.t, self.net, self.on = t, net, on
        if on:
            n = 2 * ((t.B + 1) // 2)
            w = getattr(buf, "norm_words", None)
            if w is None or w.numel() != n or w.device != t.device:
                buf.norm_words = torch.ones(n, dtype=torch.int32, device=t.device)
            self.words = buf.norm_words

    def __enter__(self):
        if self.on:
            self.net.norm_out = self.words
            self.t.set_norm_words(self.words)
        return self

    def __exit__(self, *exc):
        if self.on:
            self.net.norm_out = None
            self.t.set_norm_words(None)
        return False


def _native_trunk(net, buf):
    """the step net runs the lzm_conv_trunk kernel straight on the latent pool"""
    return getattr(net, "native", None) is not None and tuple(buf.pool.shape[2:]) == (64, 8, 8)


class MuZeroMCTSCtree(object):
    """MCTS for MuZero on the GPU (reference: mcts_ctree.py:172-321)."""

    config = dict(
        root_dirichlet_alpha=0.3,
        root_noise_weight=0.25,
        pb_c_base=19652,
        pb_c_init=1.25,
        value_delta_max=0.01,
        env_type='not_board_games',
    )

    @classmethod
    def default_config(cls: type) -> EasyDict:
        cfg = EasyDict(copy.deepcopy(cls.config))
        cfg.cfg_type = cls.__name__ + 'Dict'
        return cfg

    def __init__(self, cfg: EasyDict = None) -> None:
        default_config = self.default_config()
        default_config.update(cfg)
        self._cfg = default_config
        self.inverse_scalar_transform_handle = InverseScalarTransform(
            self._cfg.model.support_scale, self._cfg.device, self._cfg.model.categorical_distribution
        )
        self._buf = _SearchBuffers()
        self._graphs = _GraphCache(int(self._cfg.get('graph_cache_size', 4)))
        self._packed = PackedCache()
        self._folded = FoldedCache()

    # 'glibc': the reference's tie-break stream, bit-exact (default); 'philox': independent
    # counter-based stream per root (LZM_RNG_FAST), no batch-serial dependency.
    rng_mode = 'glibc'

    @classmethod
    def roots(cls: int, active_collect_env_num: int, legal_actions: List[Any]) -> "mz_tree.Roots":
        return mz_tree.Roots(active_collect_env_num, legal_actions, fast_rng=(cls.rng_mode == 'philox'))

    @classmethod
    def roots_from_mask(cls, action_mask: torch.Tensor) -> "mz_tree.Roots":
        """roots() with the legal lists taken from a device action mask (no host round trip)"""
        return mz_tree.Roots.from_action_mask(action_mask, fast_rng=(cls.rng_mode == 'philox'))

    def _categorical(self):
        return bool(self._cfg.model.get('categorical_distribution', True))

    def _fused(self, model, t):
        """(packed weights, dims) when the whole search can run as one lzm_search_mlp launch:
        a MuZeroModelMLP-shaped network with categorical heads, eval-mode BatchNorm and ReLU."""
        if not self._cfg.get('fused_search', True) or not self._categorical() or t.ez:
            return None
        try:
            packed, dims = self._packed.get(model, t.device)
        except NotPackable:
            return None
        if dims["actions"] != t.A or dims["support"] != 2 * int(self._cfg.model.support_scale) + 1:
            return None
        return packed, dims

    def _fused_conv(self, model, t, shape):
        """The native split-precision FoldedConvNet when the whole search can run as one lzm_search_conv
        launch (conv MuZeroModel, 64 x 8 x 8 latent, packed heads with K multiples of 128, one workgroup
        per root, up to 1024 roots: past the CU count they queue); None otherwise (the generic
        per-simulation path). cfg.fused_search (default on) and
        LZM_FUSED_CONV=0 turn it off."""
        if not self._cfg.get('fused_search', True) or t.ez or os.environ.get("LZM_FUSED_CONV", "1") == "0":
            return None
        if tuple(shape) != (64, 8, 8) or t.B > 1024:  # (lzm_search_conv: kScMaxRoots)
            return None
        net = _step_net(self, model)
        hp = getattr(net, "heads", None)
        if getattr(net, "native", None) is None or hp is None or getattr(net, "precision", None) != "split" \
                or getattr(net, "ez", True):
            return None
        if hp["Kr"] % 128 or hp["Khd"] % 128 or hp["off_policy"] % 128 or hp["A"] != t.A:
            return None
        return net

    def _loop(self, t, model, buf, mm, vtp_in, seeds, S, row, rec=None, infer=None, net=None):
        """The S simulations (mcts_ctree.py:255-321), all enqueued on the current stream.
        infer: optional device int64 [S], per simulation the number of roots that ran inference
        (search-with-reuse: roots whose walk stopped on an expanded node report x = -1).
        net: the step network to run (default: _step_net(model))."""
        cfg = self._cfg
        disc = float(np.float32(cfg.discount_factor))
        cat = self._categorical()
        new_minmax(t.B, cfg.value_delta_max, t.device, out=mm)
        model = _step_net(self, model) if net is None else net
        native = _native_trunk(model, buf)
        with _HeadVerdicts(t, model, buf, native and cat and getattr(model, "heads", None) is not None):
            self._sims(t, model, buf, mm, vtp_in, seeds, S, row, rec, infer, native, cat, disc)

    def _sims(self, t, model, buf, mm, vtp_in, seeds, S, row, rec, infer, native, cat, disc):
        cfg = self._cfg
        fuse = _fuse_traverse(cfg, t)
        for k in range(S):
            if k == 0 or not fuse:
                t.traverse(mm, seeds[k:k + 1], vtp_in, int(cfg.pb_c_base), float(cfg.pb_c_init), disc)
            if infer is not None:
                infer[k] = (t.x >= 0).sum()
            if native:  # leaf latents read from the pool and the next latents filed by the trunk kernel
                out = model.step_from_pool(buf.pool, t.x, t.action, buf.pool[k + 1], range_err=t.error_word(4))
            else:
                t.gather(buf.pool, row, buf.net_in)
                out = model.recurrent_inference(buf.net_in, t.action64)
            logits = out.policy_logits.float().contiguous()
            if rec is not None:
                rec.step(k, t, logits)
            kw = dict(next_latent=None if native else out.latent_state.float().contiguous(),
                      pool_slot=None if native else buf.pool[k + 1], row_elems=0 if native else row,
                      out_decoded=None if rec is None else rec.decoded[k])
            if fuse and k + 1 < S:  # this simulation's backup and the next one's traverse in one launch
                t.decode_backprop_traverse(k + 1, disc, mm, out.reward.float().contiguous(),
                                           out.value.float().contiguous(), cat, logits, t.vtp, seeds[k + 1:k + 2],
                                           vtp_in, int(cfg.pb_c_base), float(cfg.pb_c_init), **kw)
            else:
                t.decode_backprop(k + 1, disc, mm, out.reward.float().contiguous(), out.value.float().contiguous(),
                                  cat, logits, t.vtp, **kw)

    def search(self, roots: Any, model: torch.nn.Module, latent_state_roots: List[Any],
               to_play_batch: Union[int, List[Any]], seeds: torch.Tensor = None, step: dict = None) -> None:
        """seeds (not in the reference): optional device int32 [num_simulations] traverse seeds
        (the srand(tv_usec) values, uint32 bits) instead of the host seed source — keeps the call
        free of host copies (HIP-graph capture, lightzero_amd.collect).
        step (not in the reference; lightzero_amd.collect): dict(count=int64 device counter,
        base=int, dist=int32 [B, A], values=float32 [B], increment=True) — the collect step's glue
        in the search itself: seeds (base + count * S + k) mod 10^6 (`seeds` ignored), count
        incremented (unless increment=False), the
        root outputs (get_distributions / get_values as device tensors) written to dist / values,
        fresh min-max bounds. The one-launch search does all of it in its kernel
        (lzm_search_set_step); other paths run the same steps as separate launches."""
        with torch.no_grad():
            model.eval()
            t = roots.tree
            if t is None:
                raise RuntimeError("search: roots must be prepared (Roots.prepare / prepare_no_noise) first")
            B, S = roots.num, int(self._cfg.num_simulations)
            t.reserve(S)
            t.set_pb_c(int(self._cfg.pb_c_base), float(self._cfg.pb_c_init))
            dev = t.device
            lat0 = _latent_tensor(latent_state_roots, dev)
            shape = lat0.shape[1:]
            row = int(np.prod(shape)) if len(shape) else 1
            rec = _Recorder(S, B, t.A, dev) if getattr(self, "record", False) else None
            fz = self._fused(model, t)
            cz = self._fused_conv(model, t, shape) if fz is None else None
            graph = fz is None and cz is None and rec is None and self._cfg.get('use_hip_graph', False)
            gkey = _graph_key(t, model, B, S, shape) if graph else None
            entry = self._graphs.get(gkey, model, t) if graph else None
            # a captured search owns its buffers (they are what its kernels point at)
            buf = entry.buf if entry is not None else (_SearchBuffers() if graph else self._buf).get(B, S, shape, dev)
            if lat0.data_ptr() != buf.pool[0].data_ptr():  # (the collect step writes it in place)
                buf.pool[0].copy_(lat0.reshape((B,) + tuple(shape)))
            # the one-launch searches read device seeds / to_play in place (no staging copies)
            in_place = (fz is not None or cz is not None) and rec is None
            # the one-launch searches run the collect step's glue in their kernels (lzm_search_set_step:
            # seeds from the step counter, fresh min-max bounds, root outputs, the counter increment)
            step_in_kernel = step is not None and in_place
            vt = to_play_batch if in_place and _usable_i32(to_play_batch, B, dev) else None
            if vt is None:
                buf.vtp_in.copy_(_to_play_tensor(to_play_batch, B, dev))
                vt = buf.vtp_in
            sd = None
            if step is not None and not step_in_kernel:
                _lib.call("lzm_seed_sequence", _lib.ptr(step["count"]), int(step["base"]), S, _lib.ptr(buf.seeds),
                          _lib.stream_ptr())
                sd = buf.seeds
            elif step is None:
                sd = seeds if in_place and _usable_i32(seeds, S, dev) else None
                if sd is None:
                    buf.seeds.copy_(_seeds(S, dev) if seeds is None else seeds.reshape(S))
                    sd = buf.seeds
            if rec is not None:
                rec.seeds = buf.seeds.cpu().numpy().view(np.uint32)
            if cz is not None:
                # the conv network's whole search in one launch (lzm_search_conv)
                cfg = self._cfg
                if step_in_kernel:
                    t.set_step(step["count"], int(step["base"]), step.get("increment", True), step["dist"],
                               step["values"], True, cfg.value_delta_max)
                else:
                    new_minmax(B, cfg.value_delta_max, dev, out=buf.mm)
                try:
                    t.search_conv(cz, S, buf.mm, sd, vt, buf.pool, int(cfg.pb_c_base), float(cfg.pb_c_init),
                                  float(np.float32(cfg.discount_factor)), self._categorical(), rec=rec)
                finally:
                    if step_in_kernel:
                        t.set_step()
            elif fz is not None:
                packed, dims = fz
                cfg = self._cfg
                if step_in_kernel:
                    t.set_step(step["count"], int(step["base"]), step.get("increment", True), step["dist"],
                               step["values"], True, cfg.value_delta_max)
                else:
                    new_minmax(B, cfg.value_delta_max, dev, out=buf.mm)
                try:
                    t.search_mlp(dims, packed, S, buf.mm, sd, vt, buf.pool, int(cfg.pb_c_base),
                                 float(cfg.pb_c_init), float(np.float32(cfg.discount_factor)), rec=rec)
                finally:
                    if step_in_kernel:
                        t.set_step()
            elif graph:
                if entry is None:
                    entry = self._capture(t, model, buf, S, row)
                    self._graphs.put(gkey, entry)
                entry.replay()
            else:
                self._loop(t, model, buf, buf.mm, buf.vtp_in, buf.seeds, S, row, rec)
            if step is not None and not step_in_kernel:
                _lib.call("lzm_get_root_outputs", t.h, _lib.ptr(step["dist"]), _lib.ptr(step["values"]),
                          _lib.stream_ptr())
                if step.get("increment", True):
                    step["count"].add_(1)
            t.searched()
            self.last_path = "fused-conv" if cz is not None else ("fused-mlp" if fz is not None else "generic")
            roots._last_minmax = buf.mm
            self.last_record = rec

    def search_with_reuse(self, roots: Any, model: torch.nn.Module, latent_state_roots: List[Any],
                          to_play_batch: Union[int, List[Any]], true_action_list=None, reuse_value_list=None,
                          seeds: torch.Tensor = None):
        """ReZero search with value reuse (mcts_ctree.py:323-420; arXiv 2404.16364): at the root the
        true action's child is scored with the reuse value (carm_score) and choosing it ends the
        walk; roots stopping on an already expanded node skip the network and back up their reuse
        value, roots stopping at the unexpanded true-action child are expanded but back up the
        reuse value too. Runs the generic device loop with the reuse inputs on the tree handle
        (lzm_set_reuse); the network is evaluated for every root (rows of skipped roots unused).
        Returns (length, average_infer) as the reference: roots that ran inference in the last
        simulation, and inferences per simulation."""
        if true_action_list is None or reuse_value_list is None:
            raise TypeError("search_with_reuse needs true_action_list and reuse_value_list")
        with torch.no_grad():
            model.eval()
            t = roots.tree
            if t is None:
                raise RuntimeError("search_with_reuse: roots must be prepared (Roots.prepare / prepare_no_noise) first")
            if t.fast_rng:
                raise ValueError("search_with_reuse: parity (glibc) mode only")
            B, S = roots.num, int(self._cfg.num_simulations)
            t.reserve(S)
            t.set_pb_c(int(self._cfg.pb_c_base), float(self._cfg.pb_c_init))
            dev = t.device
            lat0 = _latent_tensor(latent_state_roots, dev)
            shape = lat0.shape[1:]
            row = int(np.prod(shape)) if len(shape) else 1
            buf = self._buf.get(B, S, shape, dev)
            buf.pool[0].copy_(lat0.reshape((B,) + tuple(shape)))
            buf.vtp_in.copy_(_to_play_tensor(to_play_batch, B, dev))
            buf.seeds.copy_(_seeds(S, dev) if seeds is None else seeds.reshape(S))
            ta = torch.as_tensor(np.asarray(true_action_list, np.int32).reshape(B) if not torch.is_tensor(
                true_action_list) else true_action_list, device=dev)
            rv = torch.as_tensor(np.asarray(reuse_value_list, np.float32).reshape(B) if not torch.is_tensor(
                reuse_value_list) else reuse_value_list, device=dev)
            rec = _Recorder(S, B, t.A, dev) if getattr(self, "record", False) else None
            if rec is not None:
                rec.seeds = buf.seeds.cpu().numpy().view(np.uint32)
            infer = torch.zeros(S, dtype=torch.int64, device=dev)
            t.set_reuse(ta, rv)
            try:
                self._loop(t, model, buf, buf.mm, buf.vtp_in, buf.seeds, S, row, rec, infer=infer)
            finally:
                t.set_reuse(None)
            roots._last_minmax = buf.mm
            self.last_record = rec
            counts = infer.cpu().numpy()
        return int(counts[-1]) if S else 0, float(counts.sum()) / max(S, 1)

    def _capture(self, t, model, buf, S, row):
        """Captures the whole S-simulation loop as one HIP graph over `buf` (the static buffers
        filled just before) and the network _step_net picks now; the entry keeps both alive."""
        net = _step_net(self, model)
        # warm up every kernel and library handle on a scratch tree (must not touch `t`)
        scratch = DeviceTree(t.B, t.A, max(S, t.sims_capacity), ez=t.ez, fast_rng=t.fast_rng, device=t.device)
        scratch.copy_roots_from(t)
        scratch.set_pb_c(int(self._cfg.pb_c_base), float(self._cfg.pb_c_init))
        self._loop(scratch, model, buf, buf.mm, buf.vtp_in, buf.seeds, S, row, net=net)
        torch.cuda.synchronize(t.device)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._loop(t, model, buf, buf.mm, buf.vtp_in, buf.seeds, S, row, net=net)
        scratch.close()
        return _GraphEntry(g, buf, net if net is not model else None, model, t)


class EfficientZeroMCTSCtree(object):
    """MCTS for EfficientZero on the GPU (reference: mcts_ctree.py:623-827)."""

    config = dict(
        root_dirichlet_alpha=0.3,
        root_noise_weight=0.25,
        pb_c_base=19652,
        pb_c_init=1.25,
        value_delta_max=0.01,
        env_type='not_board_games',
    )

    @classmethod
    def default_config(cls: type) -> EasyDict:
        cfg = EasyDict(copy.deepcopy(cls.config))
        cfg.cfg_type = cls.__name__ + 'Dict'
        return cfg

    def __init__(self, cfg: EasyDict = None) -> None:
        default_config = self.default_config()
        default_config.update(cfg)
        self._cfg = default_config
        self.inverse_scalar_transform_handle = InverseScalarTransform(
            self._cfg.model.support_scale, self._cfg.device, self._cfg.model.categorical_distribution
        )
        self._buf = _SearchBuffers()
        self._graphs = _GraphCache(int(self._cfg.get('graph_cache_size', 4)))
        self._folded = FoldedCache()

    rng_mode = 'glibc'

    @classmethod
    def roots(cls: int, active_collect_env_num: int, legal_actions: List[Any]) -> "ez_tree.Roots":
        return ez_tree.Roots(active_collect_env_num, legal_actions, fast_rng=(cls.rng_mode == 'philox'))

    def _fused_conv(self, model, t, shape, Hl):
        """The native split-precision FoldedConvNet (with the fused LSTM step packed) when the whole search
        can run as one lzm_search_conv_ez launch: conv EfficientZeroModel, 64 x 8 x 8 latent, head K
        multiples of 128, LSTM width a multiple of 128, max(B, 2 T) workgroups co-resident (T = ceil(B / 64)
        * H / 16 LSTM tiles); None otherwise (the generic per-simulation path). cfg.fused_search (default
        on) and LZM_FUSED_CONV=0 turn it off."""
        if not self._cfg.get('fused_search', True) or not t.ez or os.environ.get("LZM_FUSED_CONV", "1") == "0":
            return None
        if tuple(shape) != (64, 8, 8) or Hl % 128 or Hl > 1024 or Hl // 16 > 64:
            return None
        tiles = -(-t.B // 64) * (Hl // 16)
        if t.B > 256 or max(t.B, 2 * tiles) > _device_cus(t.device):
            return None
        net = _step_net(self, model)
        hp = getattr(net, "heads", None)
        if getattr(net, "native", None) is None or hp is None or getattr(net, "precision", None) != "split" \
                or not getattr(net, "ez", False) or getattr(net, "lstm_frag", None) is None:
            return None
        if hp["Khd"] % 128 or hp["off_policy"] % 128 or hp["A"] != t.A or hp["Kr"] != Hl \
                or (net.r_ch * 64 + Hl) % 128:
            return None
        return net

    def _loop(self, t, model, buf, S, row, Hl, rec=None, net=None, infer=None):
        """The S simulations (mcts_ctree.py:756-827), all enqueued on the current stream. infer: optional
        device int64 [S], per simulation the number of roots that ran inference (search-with-reuse)."""
        cfg = self._cfg
        disc = float(np.float32(cfg.discount_factor))
        horizon = int(cfg.lstm_horizon_len)
        cat = bool(cfg.model.get('categorical_distribution', True))
        B = t.B
        new_minmax(B, cfg.value_delta_max, t.device, out=buf.mm)
        model = _step_net(self, model) if net is None else net
        native = _native_trunk(model, buf)
        with _HeadVerdicts(t, model, buf, native and cat and getattr(model, "heads", None) is not None):
            self._sims(t, model, buf, S, row, Hl, rec, native, cat, disc, horizon, infer)

    def _sims(self, t, model, buf, S, row, Hl, rec, native, cat, disc, horizon, infer=None):
        cfg = self._cfg
        B = t.B
        fuse = _fuse_traverse(cfg, t) and infer is None
        for k in range(S):
            if k == 0 or not fuse:
                t.traverse(buf.mm, buf.seeds[k:k + 1], buf.vtp_in, int(cfg.pb_c_base), float(cfg.pb_c_init), disc)
            if infer is not None:
                infer[k] = (t.x >= 0).sum()
            if native:
                # the LSTM state is gathered from / filed (reset-masked) into the state pools on the device
                out = model.step_from_pool_lstm(buf.pool, t.x, t.action, buf.pool[k + 1], buf.extra[0], buf.extra[1],
                                                k, t.search_len, horizon, err=t.error_word(3),
                                                range_err=t.error_word(4))
            else:
                t.gather(buf.extra[0], Hl, buf.extra_in[0])
                t.gather(buf.extra[1], Hl, buf.extra_in[1])
                hidden = (buf.extra_in[0].unsqueeze(0), buf.extra_in[1].unsqueeze(0))
                t.gather(buf.pool, row, buf.net_in)
                out = model.recurrent_inference(buf.net_in, hidden, t.action64)
            logits = out.policy_logits.float().contiguous()
            if rec is not None:
                rec.step(k, t, logits)
            kw = dict(lstm_horizon=horizon, out_is_reset=t.is_reset,
                      next_latent=None if native else out.latent_state.float().contiguous(),
                      pool_slot=None if native else buf.pool[k + 1], row_elems=0 if native else row,
                      out_decoded=None if rec is None else rec.decoded[k])
            if fuse and k + 1 < S:  # this simulation's backup and the next one's traverse in one launch
                t.decode_backprop_traverse(k + 1, disc, buf.mm, out.value_prefix.float().contiguous(),
                                           out.value.float().contiguous(), cat, logits, t.vtp, buf.seeds[k + 1:k + 2],
                                           buf.vtp_in, int(cfg.pb_c_base), float(cfg.pb_c_init), **kw)
            else:
                t.decode_backprop(k + 1, disc, buf.mm, out.value_prefix.float().contiguous(),
                                  out.value.float().contiguous(), cat, logits, t.vtp, **kw)
            if rec is not None:
                rec.is_reset[k].copy_(t.is_reset)
            if native:
                continue  # lzm_ez_lstm_cell already filed the masked state
            # reset the LSTM state of roots whose search_len % horizon == 0 (mcts_ctree.py:810-816)
            keep = (1 - t.is_reset).to(torch.float32).unsqueeze(1)
            hc, hh = out.reward_hidden_state
            torch.mul(hc.reshape(B, Hl).float(), keep, out=buf.extra[0][k + 1])
            torch.mul(hh.reshape(B, Hl).float(), keep, out=buf.extra[1][k + 1])

    def search(self, roots: Any, model: torch.nn.Module, latent_state_roots: List[Any],
               reward_hidden_state_roots: List[Any], to_play_batch: Union[int, List[Any]],
               seeds: torch.Tensor = None, step: dict = None) -> None:
        """seeds: optional device int32 [num_simulations] traverse seeds; step: the collect step's glue
        (lightzero_amd.collect: device seeds from a step counter, root outputs into device tensors, the
        counter advanced) — both as in MuZeroMCTSCtree.search, here as small launches around the search."""
        with torch.no_grad():
            model.eval()
            t = roots.tree
            if t is None:
                raise RuntimeError("search: roots must be prepared (Roots.prepare / prepare_no_noise) first")
            B, S = roots.num, int(self._cfg.num_simulations)
            t.reserve(S)
            t.set_pb_c(int(self._cfg.pb_c_base), float(self._cfg.pb_c_init))
            dev = t.device
            if int(self._cfg.lstm_horizon_len) <= 0:
                raise ValueError("lstm_horizon_len must be > 0 (mcts_ctree.py:809)")
            lat0 = _latent_tensor(latent_state_roots, dev)
            shape = lat0.shape[1:]
            row = int(np.prod(shape)) if len(shape) else 1
            hc0 = _latent_tensor(reward_hidden_state_roots[0], dev).reshape(B, -1)
            hh0 = _latent_tensor(reward_hidden_state_roots[1], dev).reshape(B, -1)
            Hl = hc0.shape[1]
            rec = None
            graph = self._cfg.get('use_hip_graph', False) and not getattr(self, "record", False) \
                and self._fused_conv(model, t, shape, Hl) is None
            gkey = _graph_key(t, model, B, S, shape, (Hl, Hl)) if graph else None
            entry = self._graphs.get(gkey, model, t) if graph else None
            buf = entry.buf if entry is not None else (_SearchBuffers() if graph else self._buf).get(
                B, S, shape, dev, extra=(Hl, Hl))
            if lat0.data_ptr() != buf.pool[0].data_ptr():  # (the collect step writes it in place)
                buf.pool[0].copy_(lat0.reshape((B,) + tuple(shape)))
            buf.extra[0][0].copy_(hc0)
            buf.extra[1][0].copy_(hh0)
            buf.vtp_in.copy_(_to_play_tensor(to_play_batch, B, dev))
            cz = self._fused_conv(model, t, shape, Hl)
            recording = getattr(self, "record", False)
            # the one-launch search runs the collect step's glue in its kernel (lzm_search_set_step: seeds
            # from the step counter, fresh min-max bounds, root outputs, the counter increment)
            step_in_kernel = step is not None and cz is not None and not recording

            def step_seeds():  # seeds (base + count * S + k) mod 10^6 on the device
                _lib.call("lzm_seed_sequence", _lib.ptr(step["count"]), int(step["base"]), S, _lib.ptr(buf.seeds),
                          _lib.stream_ptr())

            if step is None:
                buf.seeds.copy_(_seeds(S, dev) if seeds is None else seeds.reshape(S))
            elif not step_in_kernel:
                step_seeds()
            if recording:
                rec = _Recorder(S, B, t.A, dev)
                rec.is_reset = torch.zeros((S, B), dtype=torch.int32, device=dev)
                rec.seeds = buf.seeds.cpu().numpy().view(np.uint32)
            if cz is not None:
                # the conv network's whole search, reward LSTM included, in one launch (lzm_search_conv_ez);
                # the launch needs its whole grid co-resident: when the occupancy bound refuses it, nothing
                # ran and the generic per-simulation path runs instead — eagerly only: inside a stream
                # capture the refusal is raised (the caller captures a different graph, not a fallback)
                cfg = self._cfg
                if step_in_kernel:
                    t.set_step(step["count"], int(step["base"]), step.get("increment", True), step["dist"],
                               step["values"], True, cfg.value_delta_max)
                else:
                    new_minmax(B, cfg.value_delta_max, dev, out=buf.mm)
                # eager launches are checked for hand-off timeouts (another stream's kernel can hold
                # CUs the static occupancy bound counted on): the tree (and the step counter) are kept, and a
                # search whose waits timed out is discarded and re-run on the generic path
                guard = bool(cfg.get('guard_handoffs', True)) and not torch.cuda.is_current_stream_capturing()
                if guard:
                    snap = self._snapshot(t)
                    count0 = step["count"].clone() if step_in_kernel else None
                try:
                    t.search_conv_ez(cz, S, buf.mm, None if step_in_kernel else buf.seeds, buf.vtp_in, buf.pool,
                                     buf.extra[0], buf.extra[1], int(cfg.lstm_horizon_len), int(cfg.pb_c_base),
                                     float(cfg.pb_c_init), float(np.float32(cfg.discount_factor)),
                                     bool(cfg.model.get('categorical_distribution', True)), rec=rec)
                    self.last_path = "fused"
                    if guard and t.peek_errors()[0]:
                        t.copy_roots_from(snap)
                        t.reset_errors()
                        if step_in_kernel:
                            step["count"].copy_(count0)
                            t.set_step()
                            step_in_kernel = False
                            step_seeds()
                        if rec is not None:
                            rec = _Recorder(S, B, t.A, dev)
                            rec.is_reset = torch.zeros((S, B), dtype=torch.int32, device=dev)
                            rec.seeds = buf.seeds.cpu().numpy().view(np.uint32)
                        self.timeout_fallbacks = getattr(self, "timeout_fallbacks", 0) + 1
                        self.last_path = "generic (hand-off timeout)"
                        self._loop(t, model, buf, S, row, Hl, rec)
                except _lib.ResidencyError:
                    if torch.cuda.is_current_stream_capturing():
                        raise
                    if step_in_kernel:  # nothing ran: the glue as launches around the generic path
                        t.set_step()
                        step_in_kernel = False
                        step_seeds()
                    self.residency_fallbacks = getattr(self, "residency_fallbacks", 0) + 1
                    self.last_path = "generic (co-residency refused)"
                    self._loop(t, model, buf, S, row, Hl, rec)
                finally:
                    if step_in_kernel:
                        t.set_step()
            elif graph:
                self.last_path = "generic"
                if entry is None:
                    entry = self._capture(t, model, buf, S, row, Hl)
                    self._graphs.put(gkey, entry)
                entry.replay()
            else:
                self.last_path = "generic"
                self._loop(t, model, buf, S, row, Hl, rec)
            if step is not None and not step_in_kernel:
                _lib.call("lzm_get_root_outputs", t.h, _lib.ptr(step["dist"]), _lib.ptr(step["values"]),
                          _lib.stream_ptr())
                if step.get("increment", True):
                    step["count"].add_(1)
            t.searched()
            roots._last_minmax = buf.mm
            self.last_record = rec

    def _snapshot(self, t):
        """a copy of tree t (lzm_copy_tree) in a handle kept for the purpose"""
        key = (t.B, t.A, t.ez, t.fast_rng, str(t.device))
        s = getattr(self, "_snap", None)
        if s is None or s[0] != key:
            s = (key, DeviceTree(t.B, t.A, t.sims_capacity, ez=t.ez, fast_rng=t.fast_rng, device=t.device))
            self._snap = s
        s[1].reserve(t.sims_capacity)
        s[1].copy_roots_from(t)
        return s[1]

    def search_with_reuse(self, roots: Any, model: torch.nn.Module, latent_state_roots: List[Any],
                          reward_hidden_state_roots: List[Any], to_play_batch: Union[int, List[Any]],
                          true_action_list=None, reuse_value_list=None, seeds: torch.Tensor = None):
        """ReZero search with value reuse for EfficientZero (mcts_ctree.py:829-955; arXiv 2404.16364), in
        its DEFINED form: the reference builds is_reset_list over the envs that ran inference and
        cbatch_backpropagate_with_reuse then reads it by env index (ctree_efficientzero/lib/cnode.cpp:638),
        an out-of-range, misaligned read as soon as an env skips inference; here every env's leaf gets
        is_reset = search_len % lstm_horizon_len == 0 (what the reference computes when no env skips).
        Otherwise as MuZeroMCTSCtree.search_with_reuse: the true action's root child is scored with the
        reuse value, a walk stopping on it ends there (no inference when it is expanded, its reuse
        value backed up), the device loop runs every env's network row (skipped rows unused). Returns
        (length, average_infer) as the reference."""
        if true_action_list is None or reuse_value_list is None:
            raise TypeError("search_with_reuse needs true_action_list and reuse_value_list")
        with torch.no_grad():
            model.eval()
            t = roots.tree
            if t is None:
                raise RuntimeError("search_with_reuse: roots must be prepared (Roots.prepare / prepare_no_noise) first")
            if t.fast_rng:
                raise ValueError("search_with_reuse: parity (glibc) mode only")
            if int(self._cfg.lstm_horizon_len) <= 0:
                raise ValueError("lstm_horizon_len must be > 0 (mcts_ctree.py:899)")
            B, S = roots.num, int(self._cfg.num_simulations)
            t.reserve(S)
            t.set_pb_c(int(self._cfg.pb_c_base), float(self._cfg.pb_c_init))
            dev = t.device
            lat0 = _latent_tensor(latent_state_roots, dev)
            shape = lat0.shape[1:]
            row = int(np.prod(shape)) if len(shape) else 1
            hc0 = _latent_tensor(reward_hidden_state_roots[0], dev).reshape(B, -1)
            hh0 = _latent_tensor(reward_hidden_state_roots[1], dev).reshape(B, -1)
            Hl = hc0.shape[1]
            buf = self._buf.get(B, S, shape, dev, extra=(Hl, Hl))
            buf.pool[0].copy_(lat0.reshape((B,) + tuple(shape)))
            buf.extra[0][0].copy_(hc0)
            buf.extra[1][0].copy_(hh0)
            buf.vtp_in.copy_(_to_play_tensor(to_play_batch, B, dev))
            buf.seeds.copy_(_seeds(S, dev) if seeds is None else seeds.reshape(S))
            ta = torch.as_tensor(np.asarray(true_action_list, np.int32).reshape(B) if not torch.is_tensor(
                true_action_list) else true_action_list, device=dev)
            rv = torch.as_tensor(np.asarray(reuse_value_list, np.float32).reshape(B) if not torch.is_tensor(
                reuse_value_list) else reuse_value_list, device=dev)
            rec = None
            if getattr(self, "record", False):
                rec = _Recorder(S, B, t.A, dev)
                rec.is_reset = torch.zeros((S, B), dtype=torch.int32, device=dev)
                rec.seeds = buf.seeds.cpu().numpy().view(np.uint32)
            infer = torch.zeros(S, dtype=torch.int64, device=dev)
            t.set_reuse(ta, rv)
            try:
                self._loop(t, model, buf, S, row, Hl, rec, infer=infer)
            finally:
                t.set_reuse(None)
            roots._last_minmax = buf.mm
            self.last_record = rec
            counts = infer.cpu().numpy()
        return int(counts[-1]) if S else 0, float(counts.sum()) / max(S, 1)

    def _capture(self, t, model, buf, S, row, Hl):
        """The S-simulation loop captured as one HIP graph (see MuZeroMCTSCtree._capture)."""
        net = _step_net(self, model)
        scratch = DeviceTree(t.B, t.A, max(S, t.sims_capacity), ez=t.ez, fast_rng=t.fast_rng, device=t.device)
        scratch.copy_roots_from(t)
        scratch.set_pb_c(int(self._cfg.pb_c_base), float(self._cfg.pb_c_init))
        self._loop(scratch, model, buf, S, row, Hl, net=net)
        torch.cuda.synchronize(t.device)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._loop(t, model, buf, S, row, Hl, net=net)
        scratch.close()
        return _GraphEntry(g, buf, net if net is not model else None, model, t)
