"""MuZeroModelMLP.initial_inference as one HIP launch (csrc/lzm_initial.h, lzm_mlp_initial_inference).

The collect step (MuZeroPolicy._forward_collect, lzero/policy/muzero.py:617-690) runs the model's
initial_inference before every search. ``FusedInitialInference(model)`` folds the eval-mode
BatchNorms of the representation network (lzero/model/common.py:467-517: Linear, BN,
GELU(tanh), Linear, SimNorm) and of the prediction network (common.py:883-971) into their Linears
(float64 on the host, as fused.py does for the recurrent network) and evaluates both in one kernel.
It re-folds when the module's parameters or buffers change (tensor version counters), in place,
so a captured HIP graph stays valid. ``initial_inference(obs)`` returns the module's output type;
models it does not recognise raise NotPackable (callers fall back to the module).
"""
import numpy as np
import torch
import torch.nn as nn

from . import _lib
from .fused import NotPackable, _flat, _fold, _linear_bn_pairs
from .model_mlp import MZNetworkOutput


def describe_initial(model):
    """[(W, b)] x 8 in kernel order (R1 R2 P1 P2 V1 V2 Q1 Q2) and dims, or NotPackable."""
    rep = getattr(model, "representation_network", None)
    pred = getattr(model, "prediction_network", None)
    if rep is None or pred is None or not hasattr(rep, "fc_representation") or not hasattr(rep, "sim_norm"):
        raise NotPackable("not a MuZeroModelMLP representation network")
    mods = [m for m in _flat(rep.fc_representation) if not isinstance(m, (nn.Dropout, nn.Identity))]
    ok = (len(mods) == 4 and isinstance(mods[0], nn.Linear) and isinstance(mods[1], nn.BatchNorm1d)
          and isinstance(mods[2], nn.GELU) and getattr(mods[2], "approximate", "none") == "tanh"
          and isinstance(mods[3], nn.Linear))
    if not ok:
        raise NotPackable("representation is not Linear, BN, GELU(tanh), Linear")
    group = int(getattr(rep.sim_norm, "dim", 0))
    try:
        seqs = [pred.fc_prediction_common, pred.fc_value_head, pred.fc_policy_head]
    except AttributeError as e:
        raise NotPackable(f"not a PredictionNetworkMLP: {e}") from None
    groups = [_linear_bn_pairs(s) for s in seqs]
    if [[r for _, _, r in g] for g in groups] != [[True, True], [True, False], [True, False]]:
        raise NotPackable("unexpected prediction layer structure")
    layers = [_fold(mods[0], mods[1]), _fold(mods[3], None)]
    layers += [_fold(l, bn) for g in groups for (l, bn, _) in g]
    O, H = layers[0][0].shape[1], layers[0][0].shape[0]
    F, V, A = layers[4][0].shape[0], layers[5][0].shape[0], layers[7][0].shape[0]
    if group <= 0 or H % group or max(O, H, V, A) > 1024 or F > 256:
        raise NotPackable("shape outside the kernel's limits")
    return layers, dict(obs=O, hidden=H, head_hidden=F, support=V, actions=A, group=group)


class FusedInitialInference:
    def __init__(self, model):
        self.model = model
        self.key = None
        self.flat = None
        self._pack()

    def refresh(self):
        self._pack()

    def _pack(self):
        m = self.model
        ver = tuple(t._version for t in list(m.parameters()) + list(m.buffers()))
        if ver == self.key:
            return
        layers, dims = describe_initial(m)
        dev = next(m.parameters()).device
        parts, offs, o = [], [], 0
        for W, b in layers:
            wt = W.t().contiguous().reshape(-1)
            offs += [o, o + wt.numel()]
            o += wt.numel() + b.numel()
            parts += [wt, b.reshape(-1)]
        flat = torch.cat(parts).to(device=dev, dtype=torch.float32).contiguous()
        if self.flat is None or self.flat.shape != flat.shape:
            self.flat = flat
        else:
            self.flat.copy_(flat)  # in place: captured graphs keep reading this buffer
        self.offsets = np.asarray(offs, dtype=np.int64)
        self.dims = dims
        self.key = ver

    def initial_inference(self, obs, latent_out=None, prepare=None):
        """latent_out: optional float32 [B, H] (contiguous) to write the latent into (e.g. a search's
        root slot, so the search does not copy it). prepare: optional dict(roots, noise_weight, noises,
        rewards, to_play) — also Roots.prepare_device with the policy logits, in the same launch."""
        self._pack()
        d = self.dims
        x = obs.reshape(obs.shape[0], -1)
        if x.dtype != torch.float32 or not x.is_contiguous():
            x = x.float().contiguous()
        B = x.shape[0]
        if x.shape[1] != d["obs"]:
            raise ValueError(f"observation width {x.shape[1]} != {d['obs']}")
        kw = dict(dtype=torch.float32, device=x.device)
        latent = torch.empty((B, d["hidden"]), **kw) if latent_out is None else latent_out.reshape(B, d["hidden"])
        if latent_out is not None and (not latent.is_contiguous() or latent.dtype != torch.float32):
            raise ValueError("latent_out must be a contiguous float32 [B, H] tensor")
        value = torch.empty((B, d["support"]), **kw)
        policy = torch.empty((B, d["actions"]), **kw)
        if prepare is None:
            _lib.call("lzm_mlp_initial_inference", B, d["obs"], d["hidden"], d["head_hidden"], d["support"],
                      d["actions"], d["group"], _lib.ptr(x), _lib.ptr(self.flat), self.offsets.ctypes.data,
                      _lib.ptr(latent), _lib.ptr(value), _lib.ptr(policy), _lib.stream_ptr())
        else:
            t, legal, count = prepare["roots"].device_legal(d["actions"], x.device)
            noises = prepare.get("noises")
            f32 = dict(device=x.device, dtype=torch.float32)
            _lib.call("lzm_mlp_initial_inference_prepare", t.h, B, d["obs"], d["hidden"], d["head_hidden"],
                      d["support"], d["actions"], d["group"], _lib.ptr(x), _lib.ptr(self.flat),
                      self.offsets.ctypes.data, _lib.ptr(latent), _lib.ptr(value), _lib.ptr(policy), _lib.ptr(legal),
                      _lib.ptr(count), None if noises is None else _lib.ptr(noises.to(**f32).contiguous()),
                      float(prepare["noise_weight"]), _lib.ptr(prepare["rewards"].to(**f32).contiguous()),
                      _lib.ptr(prepare["to_play"].to(device=x.device, dtype=torch.int32).contiguous()),
                      _lib.stream_ptr())
        return MZNetworkOutput(value, [0. for _ in range(B)], policy, latent)


def fused_initial_or_none(model):
    try:
        return FusedInitialInference(model)
    except NotPackable:
        return None
