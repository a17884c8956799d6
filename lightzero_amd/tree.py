"""DeviceTree: one lzm_handle (a batch of search trees resident in HBM) plus its result buffers.

Host-side owner of the structures the reference keeps in ``CRoots`` + ``CSearchResults``
(/root/reference/lzero/mcts/ctree/ctree_muzero/lib/cnode.h:48-79). All tensors are on the GPU;
every method enqueues work on the current torch stream and never synchronises.
"""
import ctypes
import itertools
import threading
import time

import numpy as np
import torch

from . import _lib
from ._lib import call, ptr, stream_ptr

# ----------------------------------------------------------------------------- seeds
_seed_lock = threading.Lock()
_seed_source = None


def reference_time_seed():
    """The reference seeds every batch_traverse with gettimeofday().tv_usec (common_lib/utils.cpp:25)."""
    return int(time.time_ns() // 1000 % 1000000)


def set_seed_source(fn):
    """Install a callable returning the next traverse seed (None restores the time seed)."""
    global _seed_source
    with _seed_lock:
        _seed_source = fn


def next_seed():
    with _seed_lock:
        fn = _seed_source
    return int(fn() if fn is not None else reference_time_seed()) & 0xFFFFFFFF


class SequentialSeeds:
    """Deterministic seed source: usec_k = (1000003*seed + k) mod 1e6."""

    def __init__(self, seed):
        self.seed, self.k = int(seed), 0

    def __call__(self):
        v = (1000003 * self.seed + self.k) % 1000000
        self.k += 1
        return v


# ----------------------------------------------------------------------------- handle
_uids = itertools.count(1)


class DeviceTree:
    def __init__(self, num_roots, action_space, max_sims=64, ez=False, fast_rng=False, device=None):
        _lib.require_gpu()
        self.uid = next(_uids)  # never reused (a handle address can be, after lzm_destroy)
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.B, self.A = int(num_roots), int(action_space)
        self.ez, self.fast_rng = bool(ez), bool(fast_rng)
        flags = (_lib.LZM_TREE_EZ if ez else 0) | (_lib.LZM_RNG_FAST if fast_rng else 0)
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            call("lzm_create", self.B, self.A, int(max_sims), flags, ctypes.byref(h))
        self.h = h
        _lib.register_owner(self)  # closed at exit before the runtime's own teardown
        self.generation = 0
        self._pb_c = (19652, 1.25)  # lzm_create builds the table for the reference defaults
        i32 = dict(dtype=torch.int32, device=self.device)
        B = self.B
        self.x = torch.zeros(B, **i32)
        self.y = torch.zeros(B, **i32)
        self.action = torch.zeros(B, **i32)
        self.action64 = torch.zeros(B, dtype=torch.int64, device=self.device)
        self.vtp = torch.zeros(B, **i32)
        self.search_len = torch.zeros(B, **i32)
        self.is_reset = torch.zeros(B, **i32)
        self.seed_buf = torch.zeros(1, dtype=torch.int32, device=self.device)
        self._unchecked = False  # a search ran whose error words no getter has checked yet

    def searched(self):
        """mark that a search (or traverse) ran: the next result getter checks the error words once"""
        self._unchecked = True

    def check_once(self):
        """check_errors(clear=True) once per search, by whichever result getter runs first: raises
        LzmError when the search's tie-break stream broke (the words are cleared as they are read, so a
        pooled tree never carries them into the next owner's searches)"""
        if self._unchecked:
            self._unchecked = False
            self.check_errors(clear=True)

    def reset_errors(self, stream=None):
        """zero the sticky error words without raising (a recycled handle starts clean); synchronises"""
        out = (ctypes.c_int32 * _lib.LZM_ERR_WORDS)()
        _lib.load().lzm_check_errors(self.h, out, 1, stream_ptr(stream))
        self._unchecked = False

    @property
    def sims_capacity(self):
        return _lib.load().lzm_sims_capacity(self.h)

    def reserve(self, max_sims):
        if max_sims > self.sims_capacity:
            with torch.cuda.device(self.device):
                call("lzm_reserve", self.h, int(max_sims))
            self.generation += 1  # device buffers moved: captured graphs are stale

    def set_pb_c(self, pb_c_base, pb_c_init):
        key = (int(pb_c_base), float(np.float32(pb_c_init)))
        if key != self._pb_c:
            with torch.cuda.device(self.device):
                call("lzm_set_pb_c", self.h, key[0], key[1])
            self._pb_c = key

    def copy_roots_from(self, other, stream=None):
        call("lzm_copy_tree", self.h, other.h, stream_ptr(stream))

    def close(self):
        h = getattr(self, "h", None)
        if h is not None and h.value:
            try:
                _lib.load().lzm_destroy(h)
            except Exception:  # interpreter shutdown
                pass
        self.h = None

    def __del__(self):
        self.close()

    # -- calls ---------------------------------------------------------------------------
    def prepare(self, legal, count, noises, noise_weight, rewards, logits, to_play, stream=None):
        call("lzm_roots_prepare", self.h, ptr(legal), ptr(count), ptr(noises), float(noise_weight), ptr(rewards),
             ptr(logits), ptr(to_play), stream_ptr(stream))

    def set_norm_words(self, words=None):
        """int32 device [2 * ceil(B / 2)] ensure_softmax verdict words that the step's head kernel
        writes (lzm_conv_heads); decode_backprop then skips its own check. None restores it."""
        self._norm_words = words
        call("lzm_set_norm_words", self.h, ptr(words))

    def set_reuse(self, true_action=None, reuse_value=None):
        """ReZero search-with-reuse inputs for the following traverse / backprop calls (device int32 /
        float32 [B]; None clears). The tensors are kept alive here: the handle keeps their pointers."""
        if true_action is None:
            self._reuse = None
            call("lzm_set_reuse", self.h, None, None)
            return
        ta = true_action.to(device=self.device, dtype=torch.int32).reshape(self.B).contiguous()
        rv = reuse_value.to(device=self.device, dtype=torch.float32).reshape(self.B).contiguous()
        self._reuse = (ta, rv)
        call("lzm_set_reuse", self.h, ptr(ta), ptr(rv))

    def traverse(self, minmax, seed, vtp_in, pb_c_base=19652, pb_c_init=1.25, discount=0.997, stream=None):
        """seed: 1-element device tensor (int32/uint32 bits)."""
        self._unchecked = True
        call("lzm_traverse", self.h, int(pb_c_base), float(pb_c_init), float(discount), ptr(minmax), ptr(seed),
             ptr(vtp_in), ptr(self.x), ptr(self.y), ptr(self.action), ptr(self.action64), ptr(self.vtp),
             ptr(self.search_len), stream_ptr(stream))

    def gather(self, pool, row_elems, out, stream=None):
        call("lzm_gather_latent", self.h, ptr(pool), int(row_elems), ptr(self.x), ptr(out), stream_ptr(stream))

    def backprop(self, cur, discount, minmax, rewards, values, logits, to_play, is_reset=None, stream=None):
        call("lzm_backprop", self.h, int(cur), float(discount), ptr(minmax), ptr(rewards), ptr(values), ptr(logits),
             ptr(to_play), ptr(is_reset), stream_ptr(stream))

    def decode_backprop(self, cur, discount, minmax, reward_logits, value_logits, categorical, policy_logits, to_play,
                        lstm_horizon=0, out_is_reset=None, next_latent=None, pool_slot=None, row_elems=0,
                        out_decoded=None, stream=None):
        V = reward_logits.shape[-1] if categorical else 1
        call("lzm_decode_backprop", self.h, int(cur), float(discount), ptr(minmax), ptr(reward_logits),
             ptr(value_logits), int(V), int(bool(categorical)), ptr(policy_logits), ptr(to_play), int(lstm_horizon),
             ptr(out_is_reset), ptr(next_latent), ptr(pool_slot), int(row_elems), ptr(out_decoded), stream_ptr(stream))

    def decode_backprop_traverse(self, cur, discount, minmax, reward_logits, value_logits, categorical, policy_logits,
                                 to_play, seed, vtp_in, pb_c_base=19652, pb_c_init=1.25, lstm_horizon=0,
                                 out_is_reset=None, next_latent=None, pool_slot=None, row_elems=0, out_decoded=None,
                                 stream=None):
        """decode_backprop of simulation `cur` and the traverse of the next one in one launch (parity
        mode); the traverse outputs overwrite x / y / action / vtp / search_len."""
        V = reward_logits.shape[-1] if categorical else 1
        call("lzm_decode_backprop_traverse", self.h, int(cur), float(discount), ptr(minmax), ptr(reward_logits),
             ptr(value_logits), int(V), int(bool(categorical)), ptr(policy_logits), ptr(to_play), int(lstm_horizon),
             ptr(out_is_reset), ptr(next_latent), ptr(pool_slot), int(row_elems), ptr(out_decoded), int(pb_c_base),
             float(pb_c_init), ptr(seed), ptr(vtp_in), ptr(self.x), ptr(self.y), ptr(self.action), ptr(self.action64),
             ptr(self.vtp), ptr(self.search_len), stream_ptr(stream))

    def search_mlp(self, dims, weights, S, minmax, seeds, vtp_in, pool, pb_c_base=19652, pb_c_init=1.25,
                   discount=0.997, rec=None, stream=None):
        """One launch for the whole search (lzm_search_mlp); rec: optional _Recorder-like object."""
        r = (lambda n: None) if rec is None else (lambda n: ptr(getattr(rec, n)))
        self._unchecked = True
        call("lzm_search_mlp", self.h, dims["hidden"], dims["head_hidden"], dims["support"], int(dims["res"]),
             ptr(weights), int(S), int(pb_c_base), float(pb_c_init), float(discount), ptr(minmax), ptr(seeds),
             ptr(vtp_in), ptr(pool), r("x"), r("action"), r("search_len"), r("decoded"), r("policy_logits"),
             stream_ptr(stream))

    def search_conv(self, net, S, minmax, seeds, vtp_in, pool, pb_c_base=19652, pb_c_init=1.25, discount=0.997,
                    categorical=True, rec=None, stream=None):
        """One launch for the whole search of a conv MuZeroModel (lzm_search_conv; net: a native
        split-precision conv_infer.FoldedConvNet); rec: optional _Recorder-like object."""
        r = (lambda n: None) if rec is None else (lambda n: ptr(getattr(rec, n)))
        hp = net.heads
        self._unchecked = True
        call("lzm_search_conv", self.h, int(S), int(pb_c_base), float(pb_c_init), float(discount), ptr(minmax),
             ptr(seeds), ptr(vtp_in), ptr(pool), ptr(net.native), ptr(net.actmap), int(net.n_dres), int(net.n_pres),
             int(net.r_ch), int(net.h_ch), ptr(hp["w1t"]), ptr(hp["b1"]), ptr(hp["w2q"]), ptr(hp["b2"]), int(hp["Kr"]),
             int(hp["Khd"]), int(hp["off_policy"]), int(hp["Vr"]), int(hp["Vv"]), int(bool(categorical)), r("x"),
             r("action"), r("search_len"), r("decoded"), r("policy_logits"), stream_ptr(stream))

    def search_conv_ez(self, net, S, minmax, seeds, vtp_in, pool, hpool, cpool, horizon, pb_c_base=19652,
                       pb_c_init=1.25, discount=0.997, categorical=True, rec=None, stream=None):
        """One launch for the whole search of a conv EfficientZeroModel (lzm_search_conv_ez; net: a native
        split-precision conv_infer.FoldedConvNet with the fused LSTM step packed); hpool / cpool: the LSTM
        state pools [S + 1, B, H] with slot 0 = the roots' state; rec: optional _Recorder-like object
        (with is_reset)."""
        r = (lambda n: None) if rec is None else (lambda n: ptr(getattr(rec, n, None)))
        hp, t = net.heads, net.t
        self._unchecked = True
        call("lzm_search_conv_ez", self.h, int(S), int(pb_c_base), float(pb_c_init), float(discount), ptr(minmax),
             ptr(seeds), ptr(vtp_in), ptr(pool), ptr(hpool), ptr(cpool), int(hpool.shape[2]), int(horizon),
             ptr(net.native), ptr(net.actmap), int(net.n_dres), int(net.n_pres), int(net.r_ch), int(net.h_ch),
             ptr(net.lstm_frag), ptr(t["lstm_b"]), ptr(t["vp_s"]), ptr(t["vp_t"]), ptr(hp["w1t"]), ptr(hp["b1"]),
             ptr(hp["w2q"]), ptr(hp["b2"]), int(hp["Khd"]), int(hp["off_policy"]), int(hp["Vr"]), int(hp["Vv"]),
             int(bool(categorical)), r("x"), r("action"), r("search_len"), r("decoded"), r("policy_logits"),
             r("is_reset"), stream_ptr(stream))

    def set_step(self, count=None, base=0, increment=True, dist=None, values=None, fresh_minmax=False,
                 value_delta_max=0.0):
        """Collect-step mode of the next search_mlp calls (lzm_search_set_step; host state only):
        device seeds from the int64 step counter `count` (incremented by the search if
        `increment`), root outputs into `dist` / `values`, fresh min-max bounds. set_step() clears
        it."""
        call("lzm_search_set_step", self.h, ptr(count), int(base), int(bool(increment)), ptr(dist), ptr(values),
             int(bool(fresh_minmax)), float(np.float32(value_delta_max)))

    def error_word(self, i):
        """device address (ctypes) of sticky error word i, for kernels launched outside the handle"""
        return ctypes.c_void_p(_lib.load().lzm_error_word(self.h, int(i)))

    def check_errors(self, clear=True, stream=None):
        """Post-search integrity check (synchronises the stream): raises LzmError when a look-back
        spin timed out or a draw fell outside the coefficient table on any search path of this
        handle, i.e. when the parity-mode tie-break stream may differ from the reference's, and
        SplitRangeError when a split-fp16 network value was non-finite or out of range (word 4).
        Returns the counters otherwise (all zero)."""
        out = (ctypes.c_int32 * _lib.LZM_ERR_WORDS)()
        if clear:
            self._unchecked = False
        call("lzm_check_errors", self.h, out, int(bool(clear)), stream_ptr(stream))
        return list(out)

    def peek_errors(self, stream=None):
        """the sticky error words without raising or clearing them (synchronises the stream)"""
        out = (ctypes.c_int32 * _lib.LZM_ERR_WORDS)()
        _lib.load().lzm_check_errors(self.h, out, 0, stream_ptr(stream))
        return list(out)

    def search_diagnostics(self):
        out = torch.zeros(4, dtype=torch.int32, device=self.device)
        call("lzm_search_diagnostics", self.h, ptr(out), stream_ptr())
        return out.cpu().tolist()

    def distributions(self, stream=None):
        out = torch.empty((self.B, self.A), dtype=torch.int32, device=self.device)
        call("lzm_get_distributions", self.h, ptr(out), stream_ptr(stream))
        return out

    def values(self, stream=None):
        out = torch.empty(self.B, dtype=torch.float32, device=self.device)
        call("lzm_get_values", self.h, ptr(out), stream_ptr(stream))
        return out

    def root_outputs(self, stream=None):
        """(distributions(), values()) from one launch"""
        dist = torch.empty((self.B, self.A), dtype=torch.int32, device=self.device)
        vals = torch.empty(self.B, dtype=torch.float32, device=self.device)
        call("lzm_get_root_outputs", self.h, ptr(dist), ptr(vals), stream_ptr(stream))
        return dist, vals

    def trajectories(self, tmax=64, stream=None):
        out = torch.empty((self.B, tmax), dtype=torch.int32, device=self.device)
        call("lzm_get_trajectories", self.h, ptr(out), int(tmax), stream_ptr(stream))
        return out

    def traverse_passes(self):
        out = torch.zeros(2, dtype=torch.int32, device=self.device)
        call("lzm_last_traverse_passes", self.h, ptr(out), stream_ptr())
        return out.cpu().tolist()


def new_minmax(n, value_delta_max, device, stream=None, out=None):
    mm = torch.empty((n, 4), dtype=torch.float32, device=device) if out is None else out
    call("lzm_minmax_init", ptr(mm), int(n), float(np.float32(value_delta_max)), stream_ptr(stream))
    return mm


def seed_tensor(seed, device):
    return torch.tensor([np.uint32(seed).view(np.int32)], dtype=torch.int32, device=device)


# ----------------------------------------------------------------------------- handle pool
class TreePool:
    """Re-uses handles across searches so device pointers stay stable (graph replay)."""

    def __init__(self):
        self._free = {}
        self._lock = threading.Lock()

    def acquire(self, B, A, max_sims, ez, fast_rng, device):
        key = (B, A, ez, fast_rng, str(device))
        t = None
        with self._lock:
            lst = self._free.get(key) or []
            while lst and t is None:
                c = lst.pop()
                # a tree whose owner was reclaimed by the cyclic GC can be returned here by
                # Roots.__del__ after its own finalizer closed the handle: skip it
                if c.h is not None and c.h.value:
                    t = c
        if t is None:
            t = DeviceTree(B, A, max_sims, ez=ez, fast_rng=fast_rng, device=device)
        else:
            t.reserve(max_sims)
            # the previous owner's sticky error words must not surface in this owner's searches
            # (ADVICE r03); acquiring happens between searches, never inside a graph capture
            if not torch.cuda.is_current_stream_capturing():
                t.reset_errors()
        return t

    def release(self, t):
        if t is None or t.h is None:
            return
        key = (t.B, t.A, t.ez, t.fast_rng, str(t.device))
        with self._lock:
            self._free.setdefault(key, []).append(t)


POOL = TreePool()
