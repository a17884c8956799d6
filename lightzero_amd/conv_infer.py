"""Inference-packed recurrent step of the convolutional MuZeroModel / EfficientZeroModel (configs 3, 5).

`recurrent_inference` is what the search calls every simulation (mcts_ctree.py:291-298 /
:776-790); in eval mode every BatchNorm there is an affine map, so the packed form folds each one
into the convolution or Linear in front of it (in float64, rounded once to float32):

  dynamics (muzero_model.py:505-530 / efficientzero_model.py:526-574)
    conv3x3([latent | one-hot action planes]) + BN      -> conv3x3(latent, W_lat) + actmap[a] + b
        the action planes are constant over the 8x8 plane, so their contribution is a per-action
        [C, 8, 8] map (border cells see fewer taps), computed once per parameter version;
    + latent, ReLU; residual blocks (conv+BN folded); 1x1 reward conv + BN folded, ReLU;
    MuZero: Linear+BN folded, ReLU, Linear -> reward logits;
    EfficientZero: LSTM cell (one GEMM over [x | h] with both biases), BN1d affine, ReLU,
    Linear+BN folded, ReLU, Linear -> value-prefix logits;
  prediction (common.py:854-881)
    residual blocks; the value and policy 1x1 convs (+BN) as ONE 1x1 conv with 2x16 outputs, ReLU;
    the two 1024->32 hidden Linears (+BN) as one block-diagonal 2048->64 Linear, ReLU; the two
    output Linears.

Same outputs as the module within float32 rounding (tests/test_gpu_conv.py). `initial_inference`
(once per env step) is folded the same way by `FoldedConvInitial`: every BatchNorm of the
representation network folded into its convolution (bias, residual add and ReLU as separate passes:
MIOpen's fused convolution + ReLU launch is opt-in, LZM_MIOPEN_FUSED=1, measured 1% slower per
Breakout step). Parameters are re-folded in place when the module's tensors change (version
counters), so captured HIP graphs keep valid pointers.

On the GPU the convolutional trunk (dynamics conv, residual blocks, reward 1x1, prediction blocks,
head 1x1) is ONE hand-written HIP launch per simulation, one workgroup per env with the
activations in LDS and split-fp16 MFMA convolutions (csrc/lzm_conv.h, lzm_conv_trunk_p; each f32
operand as two fp16 terms, three products per K — f32-level error on the fp16 matrix path; the
exact-f32 MFMA kernel stays selectable, precision='f32'): it reads the leaf
latent straight from the search's latent pool and writes the next latent straight into the next
pool slot (`step_from_pool`), so the gather and the pool filing kernels disappear too. The head
MLPs (reward, value, policy; both layers, ReLUs, the EZ value-prefix BatchNorm) are ONE more
launch (csrc/lzm_heads.h, lzm_conv_heads); the EfficientZero reward LSTM (gate GEMM + cell) one
split-fp16 launch (csrc/lzm_lstm.h, lzm_ez_lstm_step). The one-launch searches (lzm_search_conv,
lzm_search_conv_ez) run all of it inside the search kernel.
"""
import os
import weakref
from collections import OrderedDict

import numpy as np
import torch
import torch.nn.functional as F

from . import _lib


class NotFoldable(Exception):
    pass


def _bn_affine(bn):
    s = bn.weight.double() / torch.sqrt(bn.running_var.double() + bn.eps)
    return s, bn.bias.double() - bn.running_mean.double() * s


def _fold(w, b, bn):
    """(weight, bias) of a conv / Linear followed by eval BatchNorm -> folded float64 pair"""
    s, t = _bn_affine(bn)
    w = w.double() * s.reshape(-1, *([1] * (w.dim() - 1)))
    b = (b.double() if b is not None else torch.zeros_like(s)) * s + t
    return w, b


def _mlp_linears(seq):
    """DI-engine MLP (model_mlp.mlp) with one hidden layer: [Linear, BN, act, Linear] -> pairs"""
    mods = list(seq)
    if len(mods) != 4 or not isinstance(mods[0], torch.nn.Linear) or not isinstance(mods[1], torch.nn.BatchNorm1d) \
            or not isinstance(mods[2], torch.nn.ReLU) or not isinstance(mods[3], torch.nn.Linear):
        raise NotFoldable("head MLP is not [Linear, BatchNorm1d, ReLU, Linear]")
    return _fold(mods[0].weight, mods[0].bias, mods[1]), (mods[3].weight.double(), mods[3].bias.double())


def _resblocks(blocks):
    out = []
    for blk in blocks:
        if getattr(blk, "res_type", "basic") != "basic" or not isinstance(blk.act, torch.nn.ReLU):
            raise NotFoldable("only basic ReLU residual blocks")
        out.append((_fold(blk.conv1.weight, None, blk.bn1), _fold(blk.conv2.weight, None, blk.bn2)))
    return out


def fold_tensors(model):
    """dict name -> float32 tensor of the packed recurrent step"""
    dyn, pred = model.dynamics_network, model.prediction_network
    if getattr(model, "state_norm", False):
        raise NotFoldable("state_norm")
    if not isinstance(dyn.norm_common, torch.nn.BatchNorm2d) or not isinstance(dyn.activation, torch.nn.ReLU):
        raise NotFoldable("BN / ReLU variant only")
    A = dyn.action_encoding_dim
    C = dyn.num_channels - A
    hw = tuple(model.latent_hw)
    t = {}
    w, b = _fold(dyn.conv.weight, None, dyn.norm_common)
    t["dyn_w"], t["dyn_b"] = w[:, :C], b
    planes = torch.zeros(A, A, *hw, dtype=torch.float64, device=w.device)
    for a in range(A):
        planes[a, a] = 1.0
    t["dyn_actmap"] = F.conv2d(planes, w[:, C:], None, padding=1) + b.reshape(1, -1, 1, 1)  # [A, C, h, w]
    for name, blocks in (("dres", dyn.resblocks), ("pres", pred.resblocks)):
        for i, ((w1, b1), (w2, b2)) in enumerate(_resblocks(blocks)):
            t[f"{name}{i}_w1"], t[f"{name}{i}_b1"], t[f"{name}{i}_w2"], t[f"{name}{i}_b2"] = w1, b1, w2, b2
    t["rw_w"], t["rw_b"] = _fold(dyn.conv1x1_reward.weight, dyn.conv1x1_reward.bias, dyn.norm_reward)
    (w1, b1), (w2, b2) = _mlp_linears(dyn.fc_reward_head)
    t["rh_w1"], t["rh_b1"], t["rh_w2"], t["rh_b2"] = w1, b1, w2, b2
    if hasattr(dyn, "lstm"):
        l = dyn.lstm
        if l.num_layers != 1 or l.bidirectional or not l.bias:
            raise NotFoldable("single-layer LSTM with biases only")
        t["lstm_w"] = torch.cat([l.weight_ih_l0.double(), l.weight_hh_l0.double()], dim=1)  # [4L, in + L]
        t["lstm_b"] = l.bias_ih_l0.double() + l.bias_hh_l0.double()
        t["vp_s"], t["vp_t"] = _bn_affine(dyn.norm_value_prefix)
    wv, bv = _fold(pred.conv1x1_value.weight, pred.conv1x1_value.bias, pred.norm_value)
    wp, bp = _fold(pred.conv1x1_policy.weight, pred.conv1x1_policy.bias, pred.norm_policy)
    t["head_w"], t["head_b"] = torch.cat([wv, wp]), torch.cat([bv, bp])
    (v1, vb1), (v2, vb2) = _mlp_linears(pred.fc_value)
    (p1, pb1), (p2, pb2) = _mlp_linears(pred.fc_policy)
    fv, fp = v1.shape[1], p1.shape[1]
    hid = torch.zeros(v1.shape[0] + p1.shape[0], fv + fp, dtype=torch.float64, device=v1.device)
    hid[:v1.shape[0], :fv] = v1
    hid[v1.shape[0]:, fv:] = p1
    t["ph_w1"], t["ph_b1"] = hid, torch.cat([vb1, pb1])
    t["v_w2"], t["v_b2"], t["p_w2"], t["p_b2"] = v2, vb2, p2, pb2
    return {k: v.float().contiguous() for k, v in t.items()}


def pack_heads(t, hv):
    """lzm_conv_heads layouts (csrc/lzm_heads.h) of the folded head MLPs (fold_tensors' t; hv: value head
    channels), or None if they do not fit the kernel: w1t [3][8][32][32][4] over the three hidden layers
    (reward from r, value / policy from the value / policy planes), w2t [32][Vr + Vv + A] (and w2q [8][N2][4],
    k4-major float4s, for the one-launch search lzm_search_conv)."""
    rw1, vw1 = t["rh_w1"], t["ph_w1"]
    Kr, fv = rw1.shape[1], hv * 64
    Khd = vw1.shape[1]
    fp = Khd - fv
    if rw1.shape[0] != 32 or vw1.shape[0] != 64 or Kr > 1024 or fv > 1024 or fp > 1024 or fp <= 0 \
            or Kr % 4 or fv % 4 or Khd > 2048:
        return None
    dev = rw1.device
    W = torch.zeros(96, 1024, dtype=torch.float32, device=dev)
    W[0:32, :Kr] = rw1
    W[32:64, :fv] = vw1[:32, :fv]
    W[64:96, :fp] = vw1[32:, fv:]
    w1t = W.reshape(3, 32, 8, 32, 4).permute(0, 2, 3, 1, 4).contiguous()  # [head][part][k4][col][4]
    b1 = torch.cat([t["rh_b1"], t["ph_b1"]]).contiguous()
    w2c = torch.cat([t["rh_w2"], t["v_w2"], t["p_w2"]], dim=0)  # [N2][32]
    w2t = w2c.t().contiguous()
    w2q = w2c.reshape(-1, 8, 4).permute(1, 0, 2).contiguous()  # [8][N2][4] (the one-launch search)
    b2 = torch.cat([t["rh_b2"], t["v_b2"], t["p_b2"]]).contiguous()
    return dict(w1t=w1t, b1=b1, w2t=w2t, w2q=w2q, b2=b2, Kr=Kr, Khd=Khd, off_policy=fv, Vr=t["rh_w2"].shape[0],
                Vv=t["v_w2"].shape[0], A=t["p_w2"].shape[0])


class FoldedConvNet:
    """recurrent_inference of a conv MuZeroModel / EfficientZeroModel with every BN folded."""

    PRECISIONS = {"f32": 0, "split": 1}  # LZM_CONV_F32 / LZM_CONV_SPLIT (include/lzmcts.h)

    def __init__(self, model, precision=None):
        """precision of the native trunk: 'split' (default: f32 operands split into two fp16 terms,
        three products per K on the fp16 matrix path, f32-level error; the EZ LSTM gate GEMM too) or
        'f32' (the exact f32 matrix path); 'bf16x3' is the split precision's former
        name; LZM_CONV_PRECISION overrides the default."""
        precision = precision or os.environ.get("LZM_CONV_PRECISION", "split")
        precision = "split" if precision == "bf16x3" else precision
        if precision not in self.PRECISIONS:
            raise ValueError(f"conv trunk precision {precision!r}: expected one of {sorted(self.PRECISIONS)}")
        self.precision = precision
        self.model = model
        self.ez = hasattr(model.dynamics_network, "lstm")
        self.A = model.dynamics_network.action_encoding_dim
        self.n_dres = len(model.dynamics_network.resblocks)
        self.n_pres = len(model.prediction_network.resblocks)
        self.hv = model.prediction_network.conv1x1_value.out_channels
        self.t = None
        self._ver = None
        self.native = None  # device weight blob of lzm_conv_trunk (GPU models with a 64x8x8 latent)
        self.lstm_frag = None  # EZ: the gate-weight fragments of lzm_ez_lstm_step and lzm_search_conv_ez
        self._lstm_ws = {}
        # EZ: the gate GEMM + cell as one split-fp16 launch (the f32 precision keeps rocBLAS + the cell
        # pass; LZM_LSTM_FUSED=0 too)
        self.lstm_fused = precision == "split" and os.environ.get("LZM_LSTM_FUSED", "1") != "0"
        self.refresh()

    def _version(self):
        m = self.model
        return tuple(x._version for x in list(m.parameters()) + list(m.buffers()))

    def refresh(self):
        ver = self._version()
        if ver == self._ver:
            return
        with torch.no_grad():
            new = fold_tensors(self.model)
            if self.t is None:
                self.t = new
            else:  # in place: graphs captured over these tensors stay valid
                for k, v in new.items():
                    self.t[k].copy_(v)
            self._pack_native()
        self._ver = ver

    def _pack_native(self):
        t = self.t
        dev = t["dyn_w"].device
        if dev.type != "cuda" or tuple(t["dyn_w"].shape) != (64, 64, 3, 3) or t["rw_w"].shape[0] > 32 \
                or t["head_w"].shape[0] > 32 or tuple(self.model.latent_hw) != (8, 8):
            return
        parts = [t["dyn_w"]]
        for name, n in (("dres", self.n_dres), ("pres", self.n_pres)):
            if name == "pres":
                parts += [t["rw_w"], t["rw_b"]]
            for i in range(n):
                parts += [t[f"{name}{i}_w1"], t[f"{name}{i}_b1"], t[f"{name}{i}_w2"], t[f"{name}{i}_b2"]]
        parts += [t["head_w"], t["head_b"]]
        raw = np.ascontiguousarray(torch.cat([p.reshape(-1) for p in parts]).cpu().numpy(), dtype=np.float32)
        L = _lib.load()
        prec = self.PRECISIONS[self.precision]
        n = L.lzm_conv_trunk_floats_p(self.n_dres, self.n_pres, prec)
        host = np.zeros(n, np.float32)
        self.r_ch, self.h_ch = int(t["rw_w"].shape[0]), int(t["head_w"].shape[0])
        _lib.check(L.lzm_conv_trunk_prepare_p(prec, self.n_dres, self.n_pres, self.r_ch, self.h_ch,
                                              raw.ctypes.data, host.ctypes.data), "lzm_conv_trunk_prepare_p")
        if prec == self.PRECISIONS["split"]:  # the dynamics conv's bias bound: max |actmap| (lzm_conv.h, "Range")
            _lib.check(L.lzm_conv_trunk_actmap_bound(self.n_dres, self.n_pres, float(t["dyn_actmap"].abs().max()),
                                                     host.ctypes.data), "lzm_conv_trunk_actmap_bound")
        blob = torch.from_numpy(host).to(dev)
        heads = self._pack_heads()
        lstm = self._pack_lstm(L)
        if self.native is None:
            self.native = blob
            self.actmap = t["dyn_actmap"]  # [A, 64, 8, 8], re-folded in place
            self.heads = heads
            self.lstm_frag = lstm
        else:
            self.native.copy_(blob)
            if lstm is not None:
                self.lstm_frag.copy_(lstm)
            if heads is not None:
                for k, v in heads.items():
                    if torch.is_tensor(v):
                        self.heads[k].copy_(v)

    def _pack_lstm(self, L):
        """lzm_ez_lstm_step's split-fp16 fragments of the LSTM gate weights [4H, K] (EZ), or None
        (MuZero, or a shape the fused gate GEMM + cell kernel does not take)."""
        if not self.ez or "lstm_w" not in self.t:
            return None
        W = self.t["lstm_w"]
        H4, K = W.shape
        n = L.lzm_ez_lstm_frag_floats(K, H4 // 4)
        if H4 % 4 or n < 0:
            return None
        host = np.zeros(n, np.float32)
        w = np.ascontiguousarray(W.detach().float().cpu().numpy())
        _lib.check(L.lzm_ez_lstm_prepare(K, H4 // 4, w.ctypes.data, host.ctypes.data), "lzm_ez_lstm_prepare")
        return torch.from_numpy(host).to(W.device)

    def _pack_heads(self):
        return pack_heads(self.t, self.hv)

    def _trunk(self, pool, x, action, out_latent, err=None):
        """lzm_conv_trunk: (reward planes [B, r_ch*64], head planes [B, h_ch*64]); next latent -> out_latent.
        err: nullable device int32 word counting envs whose split activations left their range (a tree's
        lzm_error_word(4), reported by its check_errors)"""
        B = out_latent.shape[0]
        act = action if action.dtype == torch.int32 else action.to(torch.int32)
        r = torch.empty((B, self.r_ch * 64), dtype=torch.float32, device=out_latent.device)
        h = torch.empty((B, self.h_ch * 64), dtype=torch.float32, device=out_latent.device)
        _lib.call("lzm_conv_trunk_p", self.PRECISIONS[self.precision], B, self.n_dres, self.n_pres, self.r_ch,
                  self.h_ch, _lib.ptr(self.native),
                  _lib.ptr(self.actmap), _lib.ptr(pool), _lib.ptr(x), _lib.ptr(act.contiguous()), _lib.ptr(out_latent),
                  _lib.ptr(r), _lib.ptr(h), err, _lib.stream_ptr())
        return r, h

    def step_from_pool(self, pool, x, action, out_latent, hidden=None, range_err=None):
        """The recurrent step for leaf latents pool[x[b]][b] (pool [S+1, B, 64, 8, 8]); the next latent
        is written to out_latent ([B, 64, 8, 8], e.g. the next pool slot). Native trunk only."""
        r, h = self._trunk(pool, x, action, out_latent, range_err)
        return self._heads(r, h, out_latent, hidden)

    def _lstm_workspace(self, B, H, dev):
        """split-K workspace of lzm_ez_lstm_step for batch B (zero-filled once, kept per B: captured
        graphs hold its address) and a fallback error word"""
        ws = self._lstm_ws.get(B)
        if ws is None:
            n = int(_lib.load().lzm_ez_lstm_workspace_bytes(B, H))
            ws = (torch.zeros((n + 15) // 16 * 4, dtype=torch.float32, device=dev),
                  torch.zeros(1, dtype=torch.int32, device=dev))
            self._lstm_ws[B] = ws
        return ws

    def lstm_errors(self):
        """hand-off timeouts counted by lzm_ez_lstm_step calls made without a tree's error word"""
        return sum(int(e.item()) for _, e in self._lstm_ws.values())

    def step_from_pool_lstm(self, pool, x, action, out_latent, hpool, cpool, k, search_len, horizon, err=None,
                            range_err=None):
        """EfficientZero step on the pools: leaf latent pool[x[b]][b] and LSTM state (hpool, cpool)[x[b]][b]
        ([S+1, B, H] each). The next latent goes to out_latent, the next LSTM state — zeroed where
        search_len % horizon == 0 (mcts_ctree.py:810-813) — to hpool[k + 1] / cpool[k + 1]
        (csrc/lzm_lstm.h around the rocBLAS gate GEMM; the trunk kernel writes the LSTM input rows,
        lzm_conv_trunk_xin_p). Native trunk only. err: device int32 word counting the fused LSTM
        step's hand-off timeouts (a tree's lzm_error_word(3), reported by its check_errors); range_err: the trunk's
        split-range word (lzm_error_word(4))."""
        t, P = self.t, _lib.ptr
        B, H = out_latent.shape[0], hpool.shape[2]
        Kr = self.r_ch * 64
        # the trunk writes the [reward planes | leaf hidden state] LSTM input rows itself
        xin = torch.empty((B, Kr + H), dtype=torch.float32, device=out_latent.device)
        xscale = torch.empty(B, dtype=torch.int32, device=out_latent.device)  # the rows' split scales
        hd = torch.empty((B, self.h_ch * 64), dtype=torch.float32, device=out_latent.device)
        act = action if action.dtype == torch.int32 else action.to(torch.int32)
        _lib.call("lzm_conv_trunk_xin_p", self.PRECISIONS[self.precision], B, self.n_dres, self.n_pres, self.r_ch,
                  self.h_ch, P(self.native), P(self.actmap), P(pool), P(x), P(act.contiguous()), P(out_latent),
                  P(xin), Kr + H, P(hpool), H, P(xscale), P(hd), range_err, _lib.stream_ptr())
        r = xin[:, :Kr]
        h1 = torch.empty((B, H), dtype=torch.float32, device=r.device)
        c1 = torch.empty_like(h1)
        if self.lstm_frag is not None and self.lstm_fused:
            # the gate GEMM and the cell in one launch (split-fp16 MFMA, csrc/lzm_lstm.h)
            ws, werr = self._lstm_workspace(B, H, xin.device)
            _lib.call("lzm_ez_lstm_step", B, Kr + H, H, P(xin), P(xscale), P(self.lstm_frag), P(t["lstm_b"]), P(cpool),
                      P(x), P(search_len), int(horizon), P(h1), P(c1), P(hpool[k + 1]), P(cpool[k + 1]), P(ws),
                      err if err is not None else P(werr), range_err, _lib.stream_ptr())
        else:
            gates = torch.addmm(t["lstm_b"], xin, t["lstm_w"].t())
            _lib.call("lzm_ez_lstm_cell", B, H, P(gates), P(cpool), P(x), P(search_len), int(horizon), P(h1), P(c1),
                      P(hpool[k + 1]), P(cpool[k + 1]), _lib.stream_ptr())
        return self._head_mlps(r, hd, out_latent, h1, c1)

    def initial_inference(self, obs):
        return self.model.initial_inference(obs)

    def _res(self, x, name, n):
        t = self.t
        for i in range(n):
            y = F.conv2d(x, t[f"{name}{i}_w1"], t[f"{name}{i}_b1"], padding=1).relu_()
            x = F.conv2d(y, t[f"{name}{i}_w2"], t[f"{name}{i}_b2"], padding=1).add_(x).relu_()
        return x

    def recurrent_inference(self, latent_state, *args):
        t = self.t
        if self.ez:
            hidden, action = args
        else:
            (action,), hidden = args, None
        B = latent_state.shape[0]
        if self.native is not None and latent_state.is_cuda:
            nxt = torch.empty((B, 64, 8, 8), dtype=torch.float32, device=latent_state.device)
            r, h = self._trunk(latent_state.float().contiguous(), None, action, nxt)
            return self._heads(r, h, nxt, hidden)
        x = F.conv2d(latent_state, t["dyn_w"], None, padding=1)
        x.add_(t["dyn_actmap"].index_select(0, action.reshape(-1).long())).add_(latent_state).relu_()
        nxt = self._res(x, "dres", self.n_dres)
        r = F.conv2d(nxt, t["rw_w"], t["rw_b"]).relu_().reshape(B, -1)
        p = self._res(nxt, "pres", self.n_pres)
        h = F.conv2d(p, t["head_w"], t["head_b"]).relu_().reshape(B, -1)
        return self._heads(r, h, nxt, hidden)

    def _heads(self, r, hd, nxt, hidden):
        t = self.t
        B = r.shape[0]
        if self.ez:
            h0, c0 = hidden
            h0, c0 = h0.reshape(B, -1), c0.reshape(B, -1)
            gates = torch.addmm(t["lstm_b"], torch.cat([r, h0], dim=1), t["lstm_w"].t())
            i, f, g, o = gates.chunk(4, dim=1)
            c1 = torch.sigmoid(f) * c0 + torch.sigmoid(i) * torch.tanh(g)
            h1 = torch.sigmoid(o) * torch.tanh(c1)
        else:
            h1 = c1 = None
        return self._head_mlps(r, hd, nxt, h1, c1)

    def _head_mlps(self, r, hd, nxt, h1, c1):
        """reward / value / policy MLPs (EZ: the reward head reads the LSTM output h1)"""
        t = self.t
        B = r.shape[0]
        hp = getattr(self, "heads", None)
        if hp is not None and r.is_cuda:
            # every head MLP in one launch (csrc/lzm_heads.h)
            inp = h1.contiguous() if self.ez else r
            reward = torch.empty((B, hp["Vr"]), dtype=torch.float32, device=r.device)
            value = torch.empty((B, hp["Vv"]), dtype=torch.float32, device=r.device)
            policy = torch.empty((B, hp["A"]), dtype=torch.float32, device=r.device)
            P = _lib.ptr
            _lib.call("lzm_conv_heads", B, inp.shape[1], hp["Khd"], hp["off_policy"], P(inp),
                      P(t["vp_s"]) if self.ez else None, P(t["vp_t"]) if self.ez else None, P(hd.contiguous()),
                      P(hp["w1t"]), P(hp["b1"]), P(hp["w2t"]), P(hp["b2"]), hp["Vr"], hp["Vv"], hp["A"], P(reward),
                      P(value), P(policy), P(getattr(self, "norm_out", None)), _lib.stream_ptr())
            out = _Out()
            out.latent_state, out.value, out.policy_logits = nxt, value, policy
            if self.ez:
                out.value_prefix = reward
                out.reward_hidden_state = (h1.unsqueeze(0), c1.unsqueeze(0))
            else:
                out.reward = reward
            return out
        if self.ez:
            r = torch.addcmul(t["vp_t"], h1, t["vp_s"]).relu_()
        r = F.linear(r, t["rh_w1"], t["rh_b1"]).relu_()
        reward = F.linear(r, t["rh_w2"], t["rh_b2"])
        hid = F.linear(hd, t["ph_w1"], t["ph_b1"]).relu_()
        nv = t["v_w2"].shape[1]
        value = F.linear(hid[:, :nv], t["v_w2"], t["v_b2"])
        policy = F.linear(hid[:, nv:], t["p_w2"], t["p_b2"])
        out = _Out()
        out.latent_state, out.value, out.policy_logits = nxt, value, policy
        if self.ez:
            out.value_prefix = reward
            out.reward_hidden_state = (h1.unsqueeze(0), c1.unsqueeze(0))
        else:
            out.reward = reward
        return out


class _Out:
    pass


def _basic_blocks(blocks):
    """DI-engine basic ResBlocks (BN folded) -> [(w1, b1, w2, b2)]"""
    return [(w1, b1, w2, b2) for (w1, b1), (w2, b2) in _resblocks(blocks)]


def fold_representation(model):
    """The representation network (common.py:369-465, DownSample :164-266) of a conv MuZeroModel /
    EfficientZeroModel with every eval-mode BatchNorm folded into the convolution in front of it
    (float64, rounded once to float32). Returns a list of ops for FoldedConvInitial."""
    rep = model.representation_network
    if not isinstance(rep.activation, torch.nn.ReLU):
        raise NotFoldable("ReLU representation network only")
    ops = []
    if rep.downsample:
        ds = rep.downsample_net
        if not isinstance(ds.norm1, torch.nn.BatchNorm2d):
            raise NotFoldable("BatchNorm DownSample only")
        w, b = _fold(ds.conv1.weight, None, ds.norm1)
        ops.append(("conv_relu", w, b, 2))
        ops += [("basic",) + blk for blk in _basic_blocks(ds.resblocks1)]
        db = ds.downsample_block
        if getattr(db, "res_type", None) != "downsample" or not isinstance(db.act, torch.nn.ReLU):
            raise NotFoldable("unexpected downsample block")
        w1, b1 = _fold(db.conv1.weight, None, db.bn1)
        w2, b2 = _fold(db.conv2.weight, None, db.bn2)
        ops.append(("down", w1, b1, w2, b2, db.conv3.weight.double()))
        ops += [("basic",) + blk for blk in _basic_blocks(ds.resblocks2)]
        ops.append(("avgpool",))
        ops += [("basic",) + blk for blk in _basic_blocks(ds.resblocks3)]
        if ds.observation_shape[1] == 96:
            ops.append(("avgpool",))
    else:
        if not isinstance(rep.norm, torch.nn.BatchNorm2d):
            raise NotFoldable("BatchNorm representation only")
        w, b = _fold(rep.conv.weight, None, rep.norm)
        ops.append(("conv_relu", w, b, 1))
    ops += [("basic",) + blk for blk in _basic_blocks(rep.resblocks)]
    return [tuple(x.float().contiguous() if torch.is_tensor(x) else x for x in op) for op in ops]


class FoldedConvInitial:
    """initial_inference (muzero_model.py:209-239 / efficientzero_model.py:199-233) of a conv MuZeroModel /
    EfficientZeroModel with every eval-mode BatchNorm folded: the representation network as convolutions
    with biases (no BatchNorm launches), then the prediction network exactly as FoldedConvNet folds it
    (residual blocks, the value | policy 1x1 convs as one, the two hidden Linears as one block-diagonal
    Linear). Re-folds in place when the module's tensors change. Same outputs as the module within f32
    rounding (tests/test_conv_fold.py)."""

    def __init__(self, model):
        self.model = model
        self.ez = hasattr(model.dynamics_network, "lstm")
        self._ver = None
        self.ops = None
        self.t = None
        self.native = None  # lzm_conv_resnet8_p weights of the 8 x 8 tail (GPU, 64 x 8 x 8 latents)
        self.repr_native = None  # lzm_repr_downsample weights of the DownSample stages before the tail
        self._repr_ws = {}
        self.refresh()

    def _version(self):
        m = self.model
        return tuple(x._version for x in list(m.parameters()) + list(m.buffers()))

    def refresh(self):
        ver = self._version()
        if ver == self._ver:
            return
        with torch.no_grad():
            ops = fold_representation(self.model)
            t = fold_tensors(self.model)
            if self.ops is None:
                self.ops, self.t = ops, t
            else:  # in place: captured graphs keep reading these tensors
                for old, new in zip(self.ops, ops):
                    for a, b in zip(old, new):
                        if torch.is_tensor(a):
                            a.copy_(b)
                for k, v in t.items():
                    self.t[k].copy_(v)
            self._pack_native()
        self._ver = ver

    def _tail_start(self):
        """index of the first op after the representation's last average pool when every op from there
        on is a 64-channel residual block at 8 x 8 (the split trunk's shape), else None"""
        pools = [i for i, op in enumerate(self.ops) if op[0] == "avgpool"]
        if not pools or tuple(self.model.latent_hw) != (8, 8):
            return None
        i0 = pools[-1] + 1
        tail = self.ops[i0:]
        if not tail or any(op[0] != "basic" or tuple(op[1].shape) != (64, 64, 3, 3) or tuple(op[3].shape) != (64, 64, 3, 3)
                           for op in tail):
            return None
        return i0

    def _pack_native(self):
        """the 8 x 8 tail (representation blocks, prediction blocks, head 1x1) as one lzm_conv_resnet8_p
        launch on the split-fp16 trunk kernel (LZM_CONV_INIT_NATIVE=0: the MIOpen convolutions)"""
        t = self.t
        dev = t["head_w"].device
        i0 = self._tail_start()
        n_pres = 0
        while f"pres{n_pres}_w1" in t:
            n_pres += 1
        h_ch = int(t["head_w"].shape[0])
        if dev.type != "cuda" or i0 is None or h_ch > 32 or os.environ.get("LZM_CONV_INIT_NATIVE", "1") == "0" \
                or len(self.ops) - i0 > 8 or n_pres > 8:
            return
        z = torch.zeros(64 * 64 * 9 + 64 + 1, dtype=torch.float32, device=dev)
        parts = [z[:64 * 64 * 9]]
        for op in self.ops[i0:]:
            parts += [op[1], op[2], op[3], op[4]]
        parts += [z[64 * 64 * 9:]]  # a zero 1-channel reward 1x1 (weights, bias): not run
        for i in range(n_pres):
            parts += [t[f"pres{i}_w1"], t[f"pres{i}_b1"], t[f"pres{i}_w2"], t[f"pres{i}_b2"]]
        parts += [t["head_w"], t["head_b"]]
        raw = np.ascontiguousarray(torch.cat([q.reshape(-1).float() for q in parts]).cpu().numpy(), dtype=np.float32)
        L = _lib.load()
        nb = len(self.ops) - i0
        host = np.zeros(L.lzm_conv_trunk_floats_p(nb, n_pres, 1), np.float32)
        _lib.check(L.lzm_conv_trunk_prepare_p(1, nb, n_pres, 1, h_ch, raw.ctypes.data, host.ctypes.data),
                   "lzm_conv_trunk_prepare_p")
        blob = torch.from_numpy(host).to(dev)
        if self.native is None:
            self.native = blob
        else:
            self.native.copy_(blob)  # in place: captured graphs keep reading it
        self.tail = (i0, nb, n_pres, h_ch)
        self._pack_repr(L, dev, i0)
        # the value / policy MLPs after the tail as one lzm_conv_heads launch (prediction heads only)
        heads = pack_heads(t, self.model.prediction_network.conv1x1_value.out_channels)
        if getattr(self, "heads", None) is None or heads is None:
            self.heads = heads
        else:
            for k, v in heads.items():
                if torch.is_tensor(v):
                    self.heads[k].copy_(v)  # in place: captured graphs keep reading them

    def _pack_repr(self, L, dev, i0):
        """the DownSample stages in front of the tail (conv 3x3/2 -> 32, a 32-channel block, the downsample block,
        a 64-channel block, avg pool: common.py:164-265 at 64 x 64 frames) as lzm_repr_downsample's split-fp16
        launches (csrc/lzm_repr.h); LZM_REPR_NATIVE=0: MIOpen convolutions"""
        ops = self.ops[:i0]
        kinds = [op[0] for op in ops]
        obs = tuple(self.model.representation_network.downsample_net.observation_shape) \
            if getattr(self.model.representation_network, "downsample", False) else None
        if kinds != ["conv_relu", "basic", "down", "basic", "avgpool"] or obs is None or tuple(obs[1:]) != (64, 64) \
                or not 1 <= obs[0] <= 7 or os.environ.get("LZM_REPR_NATIVE", "1") == "0":
            return
        c1, b1, d, b2 = ops[0], ops[1], ops[2], ops[3]
        shapes = [(c1[1], (32, obs[0], 3, 3)), (b1[1], (32, 32, 3, 3)), (b1[3], (32, 32, 3, 3)), (d[1], (64, 32, 3, 3)),
                  (d[3], (64, 64, 3, 3)), (d[5], (64, 32, 3, 3)), (b2[1], (64, 64, 3, 3)), (b2[3], (64, 64, 3, 3))]
        if any(tuple(w.shape) != sh for w, sh in shapes) or c1[3] != 2:
            return
        parts = [c1[1], c1[2], b1[1], b1[2], b1[3], b1[4], d[1], d[2], d[3], d[4], d[5], b2[1], b2[2], b2[3], b2[4]]
        raw = np.ascontiguousarray(torch.cat([q.reshape(-1).float() for q in parts]).cpu().numpy(), dtype=np.float32)
        host = np.zeros(L.lzm_repr_floats(), np.float32)
        _lib.check(L.lzm_repr_prepare(int(obs[0]), raw.ctypes.data, host.ctypes.data), "lzm_repr_prepare")
        blob = torch.from_numpy(host).to(dev)
        if self.repr_native is None:
            self.repr_native = blob
            self.repr_cin = int(obs[0])
        else:
            self.repr_native.copy_(blob)

    def _downsample_native(self, x):
        """obs [B, C, 64, 64] -> [B, 64, 8, 8] through lzm_repr_downsample (workspace kept per B: captured graphs
        hold its address)"""
        B = x.shape[0]
        ws = self._repr_ws.get(B)
        if ws is None:
            ws = torch.empty(int(_lib.load().lzm_repr_workspace_floats(B)), dtype=torch.float32, device=x.device)
            self._repr_ws[B] = ws
        out = torch.empty((B, 64, 8, 8), dtype=torch.float32, device=x.device)
        _lib.call("lzm_repr_downsample", B, self.repr_cin, _lib.ptr(self.repr_native), _lib.ptr(x), _lib.ptr(ws),
                  _lib.ptr(out), _lib.stream_ptr())
        return out

    # MIOpen's fused convolution + bias (+ residual) + ReLU (torch.miopen_convolution_relu /
    # _add_relu): one launch per convolution instead of a convolution, a bias add / residual add and
    # a ReLU pass. Opt-in (LZM_MIOPEN_FUSED=1): measured per Breakout collect-time step 2.863 vs
    # 2.826 ms unfused (profiles/r04/ab_breakout_miopen.txt). Checked once per process.
    _fused_ok = None

    def _fused(self, x):
        if not x.is_cuda or not hasattr(torch, "miopen_convolution_relu") or FoldedConvInitial._fused_ok is False:
            return False
        if os.environ.get("LZM_MIOPEN_FUSED", "0") != "1":
            return False
        if FoldedConvInitial._fused_ok is None:
            try:
                w = torch.randn(4, 4, 3, 3, device=x.device)
                b = torch.randn(4, device=x.device)
                z = torch.randn(1, 4, 5, 5, device=x.device)
                xi = torch.randn(1, 4, 5, 5, device=x.device)
                got = torch.miopen_convolution_add_relu(xi, w, z, 1.0, b, [1, 1], [1, 1], [1, 1], 1)
                got2 = torch.miopen_convolution_relu(xi, w, b, [1, 1], [1, 1], [1, 1], 1)
                ref = F.conv2d(xi, w, b, padding=1)
                FoldedConvInitial._fused_ok = bool(torch.allclose(got, (ref + z).relu(), rtol=1e-4, atol=1e-5) and
                                                   torch.allclose(got2, ref.relu(), rtol=1e-4, atol=1e-5))
            except (RuntimeError, TypeError, NotImplementedError):
                FoldedConvInitial._fused_ok = False
        return FoldedConvInitial._fused_ok

    @staticmethod
    def _epilogue(y, b, z=None, relu=True):
        """y = relu((y + b) + z) in place: on the GPU one HIP pass (lzm_bias_add_relu) instead of
        torch's bias, residual and ReLU passes (the same float additions, the same bits)"""
        if y.is_cuda:
            _lib.call("lzm_bias_add_relu", _lib.ptr(y), _lib.ptr(b), None if z is None else _lib.ptr(z),
                      y.shape[0], y.shape[1], y.shape[2] * y.shape[3], 1 if relu else 0, _lib.stream_ptr())
            return y
        y = y + b.reshape(1, -1, 1, 1)
        if z is not None:
            y = y.add_(z)
        return y.relu_() if relu else y

    @classmethod
    def _conv_relu(cls, x, w, b, stride, fused):
        if fused:
            return torch.miopen_convolution_relu(x, w, b, [stride, stride], [1, 1], [1, 1], 1)
        return cls._epilogue(F.conv2d(x, w, None, stride=stride, padding=1).contiguous(), b)

    @classmethod
    def _conv_add_relu(cls, x, w, z, b, fused):
        """relu(conv3x3(x, w) + b + z)"""
        if fused:
            return torch.miopen_convolution_add_relu(x, w, z, 1.0, b, [1, 1], [1, 1], [1, 1], 1)
        return cls._epilogue(F.conv2d(x, w, None, padding=1).contiguous(), b, z.contiguous())

    @classmethod
    def _basic(cls, x, w1, b1, w2, b2, fused=False):
        y = cls._conv_relu(x, w1, b1, 1, fused)
        return cls._conv_add_relu(y, w2, x, b2, fused)

    def initial_inference(self, obs, latent_out=None, prepare=None):
        """latent_out: optional [B, 64, 8, 8] f32 tensor the native tail writes the latent into (the search's
        root pool slot: no copy). prepare: optional dict(roots, noise_weight, noises, rewards, to_play) — also
        Roots.prepare_device with the policy logits, in the heads' launch (lzm_conv_heads_prepare); the caller
        checks `prepared` on the output (False: the heads ran elsewhere, prepare the roots itself)."""
        self.refresh()
        t = self.t
        x = obs.float()
        if not x.is_contiguous():
            x = x.contiguous()
        fused = self._fused(x)
        native = self.native is not None and x.is_cuda
        pre = self.ops[:self.tail[0]] if native else self.ops
        if native and self.repr_native is not None and tuple(x.shape[1:]) == (self.repr_cin, 64, 64):
            x = self._downsample_native(x)  # the DownSample stages in front of the tail, split-fp16 launches
            pre = []
        for op in pre:
            kind = op[0]
            if kind == "conv_relu":
                x = self._conv_relu(x, op[1], op[2], op[3], fused)
            elif kind == "basic":
                x = self._basic(x, *op[1:], fused=fused)
            elif kind == "down":
                _, w1, b1, w2, b2, w3 = op
                y = self._conv_relu(x, w1, b1, 2, fused)
                x = self._conv_add_relu(y, w2, F.conv2d(x, w3, None, stride=2, padding=1), b2, fused)
            else:  # avgpool (count_include_pad, as nn.AvgPool2d(3, 2, 1))
                x = F.avg_pool2d(x, kernel_size=3, stride=2, padding=1)
        B = x.shape[0]
        if native:
            # the 8 x 8 tail in one launch: representation blocks -> latent, prediction blocks, head 1x1
            _, nb, n_pres, h_ch = self.tail
            x = x.contiguous()
            latent = latent_out if latent_out is not None and tuple(latent_out.shape) == tuple(x.shape) \
                and latent_out.is_contiguous() else torch.empty_like(x)
            h = torch.empty((B, h_ch * 64), dtype=torch.float32, device=x.device)
            # (no error word: a non-finite value here reaches the root latent, whose range the search checks)
            _lib.call("lzm_conv_resnet8_p", B, nb, n_pres, h_ch, _lib.ptr(self.native), _lib.ptr(x),
                      _lib.ptr(latent), _lib.ptr(h), None, _lib.stream_ptr())
            hp = getattr(self, "heads", None)
            if hp is not None and h.shape[1] == hp["Khd"]:
                # the value / policy MLPs in one launch (lzm_conv_heads, prediction heads only)
                value = torch.empty((B, hp["Vv"]), dtype=torch.float32, device=x.device)
                policy = torch.empty((B, hp["A"]), dtype=torch.float32, device=x.device)
                P = _lib.ptr
                if prepare is not None:
                    # + the root preparation from the logits, in the same launch
                    tr, legal, count = prepare["roots"].device_legal(hp["A"], x.device)
                    f32 = dict(device=x.device, dtype=torch.float32)
                    noises = prepare.get("noises")
                    _lib.call("lzm_conv_heads_prepare", tr.h, B, hp["Khd"], hp["off_policy"], P(h), P(hp["w1t"]),
                              P(hp["b1"]), P(hp["w2t"]), P(hp["b2"]), hp["Vr"], hp["Vv"], hp["A"], P(value), P(policy),
                              P(legal), P(count), None if noises is None else P(noises.to(**f32).contiguous()),
                              float(prepare["noise_weight"]), P(prepare["rewards"].to(**f32).contiguous()),
                              P(prepare["to_play"].to(device=x.device, dtype=torch.int32).contiguous()),
                              _lib.stream_ptr())
                else:
                    _lib.call("lzm_conv_heads", B, 0, hp["Khd"], hp["off_policy"], None, None, None, P(h),
                              P(hp["w1t"]), P(hp["b1"]), P(hp["w2t"]), P(hp["b2"]), hp["Vr"], hp["Vv"], hp["A"], None,
                              P(value), P(policy), None, _lib.stream_ptr())
                out = self._output(value, policy, latent, B, obs.device)
                out.prepared = prepare is not None
                return out
        else:
            latent = x
            p = latent
            i = 0
            while f"pres{i}_w1" in t:
                p = self._basic(p, t[f"pres{i}_w1"], t[f"pres{i}_b1"], t[f"pres{i}_w2"], t[f"pres{i}_b2"], fused=fused)
                i += 1
            h = self._epilogue(F.conv2d(p, t["head_w"], None).contiguous(), t["head_b"]).reshape(B, -1)
        hid = F.linear(h, t["ph_w1"], t["ph_b1"]).relu_()
        nv = t["v_w2"].shape[1]
        value = F.linear(hid[:, :nv], t["v_w2"], t["v_b2"])
        policy = F.linear(hid[:, nv:], t["p_w2"], t["p_b2"])
        return self._output(value, policy, latent, B, obs.device)

    def _output(self, value, policy, latent, B, dev):
        if self.ez:
            from .model_conv import EZNetworkOutput
            z = torch.zeros(1, B, self.model.lstm_hidden_size, device=dev)
            return EZNetworkOutput(value, [0. for _ in range(B)], policy, latent, (z, z.clone()))
        from .model_mlp import MZNetworkOutput
        return MZNetworkOutput(value, [0. for _ in range(B)], policy, latent)


def folded_initial_or_none(model):
    """FoldedConvInitial for the conv model family, None for anything else"""
    if not hasattr(model, "latent_hw") or not hasattr(model, "representation_network"):
        return None
    try:
        return FoldedConvInitial(model)
    except (NotFoldable, AttributeError):
        return None


class FoldedCache:
    """FoldedConvNet per model (None for models it does not recognise); a small LRU keyed by model
    identity, re-folded in place when the model's parameters change (FoldedConvNet.refresh)."""

    def __init__(self, cap=4):
        self.cap = int(cap)
        self._d = OrderedDict()  # id(model) -> (model weakref, FoldedConvNet or None)

    def get(self, model):
        k = id(model)
        e = self._d.get(k)
        if e is not None and e[0]() is not model:  # a dead model's id was reused
            del self._d[k]
            e = None
        if e is None:
            try:
                net = FoldedConvNet(model) if hasattr(model, "latent_hw") else None
            except (NotFoldable, AttributeError):
                net = None
            e = (weakref.ref(model), net)
            self._d[k] = e
            while len(self._d) > self.cap:
                self._d.popitem(last=False)
        elif e[1] is not None:
            e[1].refresh()
        self._d.move_to_end(k)
        return e[1]
