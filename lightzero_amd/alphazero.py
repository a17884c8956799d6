"""Batched AlphaZero search on the device.

Mirrors ``mcts_alphazero.MCTS`` (lzero/mcts/ctree/ctree_alphazero/mcts_alphazero.cpp:19-254, bound at
:335-345): the constructor takes the same arguments (max_moves, num_simulations, pb_c_base,
pb_c_init, root_dirichlet_alpha, root_noise_weight, simulate_env) and ``get_next_action`` the same
(state_config_for_env_reset, policy_value_func, temperature, sample) -> (action, action_probs). The
difference is the batch: ``get_next_actions`` searches B TicTacToe boards at once and the
policy-value function is the network's batched ``compute_policy_value(state [n, 3, 3, 3])`` ->
(probs [n, 9], value [n] or [n, 1]) (alphazero_model.py:170-183) instead of the per-env Python
callback (policy/alphazero.py:371-380): the simulate env lives inside the kernel (lzm_az.h).

Per search: lzm_az_begin, network(roots), lzm_az_step(-1), then S x (network(leaves),
lzm_az_step(k)), lzm_az_finish; with ``graph=True`` that whole sequence is one HIP graph per batch
size. Visit counts and action_probs are identical to the reference's for the same network outputs
(tests/test_gpu_alphazero.py against tests/golden/az_*.npz). The sampled action uses a Philox draw
(the reference uses std::random_device, which has no reproducible stream).
"""
import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import call, ptr, stream_ptr

ACTIONS = 9


def _fold_bn(conv, bn):
    """eval-mode BatchNorm folded into the preceding convolution (float64, then float32)"""
    scale = bn.weight.double() / torch.sqrt(bn.running_var.double() + bn.eps)
    w = conv.weight.double() * scale.reshape(-1, *([1] * (conv.weight.dim() - 1)))
    b = conv.bias.double() if conv.bias is not None else torch.zeros_like(scale)
    b = (b - bn.running_mean.double()) * scale + bn.bias.double()
    return w.float(), b.float()


class FusedAZNet:
    """The TicTacToe AlphaZeroModel (lightzero_amd.model_az, same module structure as
    lzero/model/alphazero_model.py) packed for the fused kernels: BatchNorm folded, MFMA B-fragment
    layout (lzm_az_net_prepare). Supported: 16 channels, 1 or 2 residual blocks per network, head
    width 8, 9 actions, scalar value (the TicTacToe config); anything else raises ValueError."""

    def __init__(self, model, device="cuda"):
        m = model
        nres = len(m.rep_blocks)
        ok = (nres in (1, 2) and len(m.pred_blocks) == nres and m.conv.out_channels == 16 and m.conv.in_channels == 3
              and m.flat_v == 144 and m.flat_p == 144 and m.fc_value_head[0].out_features == 8
              and m.fc_policy_head[0].out_features == 8 and m.fc_policy_head[-1].out_features == ACTIONS
              and m.fc_value_head[-1].out_features == 1 and isinstance(m.fc_value_head[1], torch.nn.LayerNorm))
        if not ok:
            raise ValueError("fused AlphaZero kernel supports the TicTacToe AlphaZeroModel config only")
        if m.training:
            raise ValueError("fused AlphaZero kernel evaluates the network in eval mode: call model.eval()")
        self.nres = nres
        with torch.no_grad():
            parts = []
            w, b = _fold_bn(m.conv, m.norm)
            parts += [w.reshape(16, 27), b]
            for blk in list(m.rep_blocks) + list(m.pred_blocks):
                for conv, bn in ((blk.conv1, blk.bn1), (blk.conv2, blk.bn2)):
                    w, b = _fold_bn(conv, bn)
                    parts += [w.reshape(16, 144), b]
            wv, bv = _fold_bn(m.conv1x1_value, m.norm_value)
            wp, bp = _fold_bn(m.conv1x1_policy, m.norm_policy)
            parts += [torch.cat([wv.reshape(16, 16), wp.reshape(16, 16)]), torch.cat([bv, bp])]
            head = torch.zeros(2448, dtype=torch.float32)
            fv, fp = m.fc_value_head, m.fc_policy_head
            for off, t in ((0, fv[0].weight), (1152, fv[0].bias), (1160, fv[1].weight), (1168, fv[1].bias),
                           (1176, fv[3].weight), (1184, fv[3].bias), (1188, fp[0].weight), (2340, fp[0].bias),
                           (2348, fp[1].weight), (2356, fp[1].bias), (2364, fp[3].weight), (2436, fp[3].bias)):
                t = t.detach().float().cpu().reshape(-1)
                head[off:off + t.numel()] = t
            parts.append(head)
            raw = torch.cat([p.detach().float().cpu().reshape(-1) for p in parts]).contiguous()
        n = int(_lib.load().lzm_az_net_floats(nres))
        out = torch.zeros(n, dtype=torch.float32)
        call("lzm_az_net_prepare", nres, ctypes.c_void_p(raw.data_ptr()), ctypes.c_void_p(out.data_ptr()))
        self.weights = out.to(device)

    def compute_policy_value(self, state):
        """the fused network on its own: state [n, 3, 3, 3] -> (probs [n, 9], value [n, 1])"""
        st = state.reshape(-1, 27).to(torch.float32).contiguous()
        n = st.shape[0]
        probs = torch.empty((n, ACTIONS), dtype=torch.float32, device=st.device)
        value = torch.empty((n, 1), dtype=torch.float32, device=st.device)
        call("lzm_az_net_eval", self.nres, ptr(self.weights), ptr(st), n, ptr(probs), ptr(value), stream_ptr())
        return probs, value


class AlphaZeroMCTS:
    def __init__(self, max_moves=9, num_simulations=50, pb_c_base=19652, pb_c_init=1.25, root_dirichlet_alpha=0.3,
                 root_noise_weight=0.25, simulate_env=None, device="cuda", graph=False, seed=0):
        if simulate_env is not None and getattr(getattr(simulate_env, "action_space", None), "n", ACTIONS) != ACTIONS:
            raise ValueError("the device simulate env is TicTacToe (9 actions)")
        _lib.require_gpu()
        self.max_moves = int(max_moves)
        self.num_simulations = int(num_simulations)
        self.pb_c_base, self.pb_c_init = float(pb_c_base), float(pb_c_init)
        self.alpha, self.noise_weight = float(root_dirichlet_alpha), float(root_noise_weight)
        self.device = torch.device(device)
        self.use_graph = bool(graph)
        self.seed = int(seed) & 0xffffffff
        self._count = torch.zeros(1, dtype=torch.int64, device=self.device)
        self._ctx = {}  # B -> per-batch buffers (and graphs)
        self.graph_cache_size = 4  # captured graphs kept per batch size

    # ------------------------------------------------------------------ per-batch buffers
    def _buffers(self, B):
        c = self._ctx.get(B)
        if c is not None:
            return c
        nbytes = ctypes.c_int64()
        call("lzm_az_workspace_bytes", B, self.num_simulations, ctypes.byref(nbytes))
        dev = self.device
        c = dict(ws=torch.empty(int(nbytes.value), dtype=torch.uint8, device=dev),
                 boards=torch.zeros((B, ACTIONS), dtype=torch.int32, device=dev),
                 start=torch.zeros(B, dtype=torch.int32, device=dev),
                 state=torch.zeros((B, 3, 3, 3), dtype=torch.float32, device=dev),
                 visits=torch.zeros((B, ACTIONS), dtype=torch.int32, device=dev),
                 probs=torch.zeros((B, ACTIONS), dtype=torch.float64, device=dev),
                 action=torch.zeros(B, dtype=torch.int32, device=dev), graphs={})
        call("lzm_az_set_constants", B, self.num_simulations, ptr(c["ws"]), self.pb_c_base, self.pb_c_init,
             self.alpha, stream_ptr())
        self._ctx[B] = c
        return c

    def _evaluate(self, pv, c, B):
        probs, value = pv(c["state"])
        probs = probs.reshape(B, -1).to(torch.float32).contiguous()
        value = value.reshape(B).to(torch.float32).contiguous()
        if probs.shape[1] < ACTIONS:
            raise ValueError("policy must cover the 9 TicTacToe actions")
        return probs, value

    def _body(self, B, pv, temperature, sample):
        c = self._buffers(B)
        S, ws, st = self.num_simulations, ptr(c["ws"]), ptr(c["state"])
        s = stream_ptr()
        with torch.no_grad():
            call("lzm_az_begin", B, S, ws, ptr(c["boards"]), ptr(c["start"]), st, s)
            probs, value = self._evaluate(pv, c, B)
            call("lzm_az_step", B, S, ws, -1, ptr(probs), probs.shape[1], ptr(value), 1, int(bool(sample)),
                 self.noise_weight, st, s)
            for k in range(S):
                probs, value = self._evaluate(pv, c, B)
                call("lzm_az_step", B, S, ws, k, ptr(probs), probs.shape[1], ptr(value), 1, 0, 0.0, st, s)
            call("lzm_az_finish", B, S, ws, float(temperature), int(bool(sample)), self.seed, ptr(self._count),
                 ptr(c["visits"]), ptr(c["probs"]), ptr(c["action"]), s)
            self._count.add_(1)

    def _run(self, B, pv, temperature, sample):
        if not self.use_graph:
            self._body(B, pv, temperature, sample)
            return
        c = self._buffers(B)
        # a bound method is a new object on every attribute access (net.compute_policy_value):
        # key on the function and its instance, so the same callable replays its graph
        key = (id(getattr(pv, "__func__", pv)), id(getattr(pv, "__self__", None)), float(temperature), bool(sample))
        g = c["graphs"].get(key)
        if g is not None and (g[1] is not getattr(pv, "__func__", pv) or g[2] is not getattr(pv, "__self__", None)):
            del c["graphs"][key]  # ids reused by new objects
            g = None
        if g is None:
            side = torch.cuda.Stream(device=self.device)
            side.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(side):
                self._body(B, pv, temperature, sample)  # warm-up: allocator pools, lazy inits
            torch.cuda.current_stream(self.device).wait_stream(side)
            self._count.sub_(1)  # the warm-up search does not count
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._body(B, pv, temperature, sample)
            # keep the function and instance alive (the key holds their ids); bounded LRU
            c["graphs"][key] = (g, getattr(pv, "__func__", pv), getattr(pv, "__self__", None))
            while len(c["graphs"]) > self.graph_cache_size:
                c["graphs"].pop(next(iter(c["graphs"])))
        else:
            c["graphs"][key] = c["graphs"].pop(key)  # most recently used last
            g = g[0]
        g.replay()

    def search_fused(self, boards, start_player_index, net, temperature=1.0, sample=True, export_tree=False):
        """The whole search (root evaluation, S simulations with the network, finalisation) in one
        launch; net: FusedAZNet. Same outputs as get_next_actions."""
        if temperature == 0:
            raise ValueError("Temperature cannot be 0")
        b = torch.as_tensor(boards).reshape(-1, ACTIONS)
        B = int(b.shape[0])
        c = self._buffers(B)
        c["boards"].copy_(b.to(device=self.device, dtype=torch.int32))
        c["start"].copy_(torch.as_tensor(start_player_index).reshape(B).to(device=self.device, dtype=torch.int32))
        call("lzm_az_search_fused", B, self.num_simulations, ptr(c["ws"]), net.nres, ptr(net.weights), ptr(c["boards"]),
             ptr(c["start"]), int(bool(sample)), self.noise_weight, float(temperature), int(bool(sample)), self.seed,
             ptr(self._count), ptr(c["visits"]), ptr(c["probs"]), ptr(c["action"]), int(bool(export_tree)),
             stream_ptr())
        self._count.add_(1)
        return c["action"], c["probs"]

    # ------------------------------------------------------------------ public API
    def get_next_actions(self, boards, start_player_index, compute_policy_value, temperature=1.0, sample=True):
        """boards [B, 9] (or [B, 3, 3]) with 0 empty / 1 / 2 stones, start_player_index [B] (0: player 1
        to move, 1: player 2). Returns (actions int32 [B], action_probs float64 [B, 9], device tensors;
        overwritten by the next call with the same B)."""
        if temperature == 0:
            raise ValueError("Temperature cannot be 0")
        b = torch.as_tensor(boards).reshape(-1, ACTIONS)
        B = int(b.shape[0])
        c = self._buffers(B)
        c["boards"].copy_(b.to(device=self.device, dtype=torch.int32))
        c["start"].copy_(torch.as_tensor(start_player_index).reshape(B).to(device=self.device, dtype=torch.int32))
        self._run(B, compute_policy_value, temperature, sample)
        return c["action"], c["probs"]

    def last_visits(self, B):
        return self._buffers(B)["visits"]

    def get_next_action(self, state_config_for_env_reset, policy_value_func, temperature=1.0, sample=True):
        """One board, the reference's signature; policy_value_func is the batched compute_policy_value."""
        cfg = state_config_for_env_reset
        init = cfg.get("init_state")
        board = np.zeros(ACTIONS, np.int32) if init is None else np.asarray(init, np.int32).reshape(ACTIONS)
        a, p = self.get_next_actions(board[None], [int(cfg["start_player_index"])], policy_value_func, temperature,
                                     sample)
        return int(a[0].item()), p[0].tolist()

    def export_tree(self, B):
        """(visit int32 [B, cap], value_sum float32 [B, cap], first int32 [B, cap], nnodes int32 [B])"""
        c = self._buffers(B)
        cap = 1 + ACTIONS * (self.num_simulations + 1)
        out = [torch.empty((B, cap), dtype=torch.int32, device=self.device),
               torch.empty((B, cap), dtype=torch.float32, device=self.device),
               torch.empty((B, cap), dtype=torch.int32, device=self.device),
               torch.empty(B, dtype=torch.int32, device=self.device)]
        call("lzm_az_export_tree", B, self.num_simulations, ptr(c["ws"]), *[ptr(t) for t in out], stream_ptr())
        return out


MCTS = AlphaZeroMCTS
