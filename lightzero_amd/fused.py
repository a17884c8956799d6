"""Fused whole-search path for MuZeroModelMLP-shaped networks (lzm_search_mlp, include/lzmcts.h).

``pack_muzero_mlp(model)`` folds every eval-mode BatchNorm1d into the Linear in front of it
(W' = W * gamma/sqrt(var+eps), b' = (b - mean) * gamma/sqrt(var+eps) + beta) and lays the
recurrent network out as the kernel reads it: per layer W[K][N] (torch weight transposed, so a
wave's lanes read consecutive output columns) followed by bias[N]. The module structure is
the reference's (lzero/model/muzero_model_mlp.py:327-440, lzero/model/common.py:883-971): the
packer walks ``dynamics_network.fc_dynamics(_1|_2)``, ``fc_reward_head`` and
``prediction_network.fc_{prediction_common,value_head,policy_head}`` and accepts any nesting of
Linear / BatchNorm1d / ReLU inside them (DI-engine's MLP nests fc blocks).
"""
import weakref
from collections import OrderedDict

import torch
import torch.nn as nn

from . import _lib


class NotPackable(Exception):
    pass


_LEAVES = (nn.Linear, nn.BatchNorm1d, nn.ReLU, nn.GELU, nn.Tanh, nn.Sigmoid, nn.LeakyReLU, nn.ELU, nn.Dropout,
           nn.Identity)


def _flat(m):
    # forward order, repeats kept (one activation instance is often shared by every layer)
    if isinstance(m, _LEAVES):
        yield m
        return
    for c in m._modules.values():
        if c is not None:
            yield from _flat(c)


def _linear_bn_pairs(seq):
    """[(Linear, BN or None, relu_after)] in forward order."""
    mods = [m for m in _flat(seq) if not isinstance(m, (nn.Dropout, nn.Identity))]
    out = []
    i = 0
    while i < len(mods):
        m = mods[i]
        if not isinstance(m, nn.Linear):
            raise NotPackable(f"unexpected {type(m).__name__} before a Linear")
        bn, act = None, None
        j = i + 1
        if j < len(mods) and isinstance(mods[j], nn.BatchNorm1d):
            bn = mods[j]
            j += 1
        if j < len(mods) and not isinstance(mods[j], (nn.Linear, nn.BatchNorm1d)):
            act = mods[j]
            j += 1
        if act is not None and not isinstance(act, nn.ReLU):
            raise NotPackable(f"activation {type(act).__name__} (fused kernel implements ReLU)")
        out.append((m, bn, act is not None))
        i = j
    return out


def _fold(lin, bn):
    W = lin.weight.detach().to(torch.float64)
    b = lin.bias.detach().to(torch.float64) if lin.bias is not None else torch.zeros(W.shape[0], dtype=torch.float64,
                                                                                      device=W.device)
    if bn is not None:
        if bn.training:
            raise NotPackable("BatchNorm in training mode")
        s = bn.weight.detach().double() / torch.sqrt(bn.running_var.detach().double() + bn.eps)
        W = W * s[:, None]
        b = (b - bn.running_mean.detach().double()) * s + bn.bias.detach().double()
    return W.float(), b.float()


def describe(model):
    """Returns (layers [(W, b, relu)], dims dict) or raises NotPackable."""
    dyn = getattr(model, "dynamics_network", None)
    pred = getattr(model, "prediction_network", None)
    if dyn is None or pred is None:
        raise NotPackable("not a MuZero model (no dynamics_network / prediction_network)")
    res = bool(getattr(dyn, "res_connection_in_dynamics", False))
    if getattr(model, "state_norm", False):
        raise NotPackable("state_norm")
    if getattr(model, "discrete_action_encoding_type", "one_hot") != "one_hot":
        raise NotPackable("non one-hot action encoding")
    try:
        seqs = [dyn.fc_dynamics_1, dyn.fc_dynamics_2] if res else [dyn.fc_dynamics]
        seqs += [dyn.fc_reward_head, pred.fc_prediction_common, pred.fc_value_head, pred.fc_policy_head]
    except AttributeError as e:  # e.g. the convolutional MuZeroModel
        raise NotPackable(f"not a MuZeroModelMLP: {e}") from None
    groups = [_linear_bn_pairs(s) for s in seqs]
    expect_relu = [[True, True]] * (2 if res else 1) + [[True, False], [True, True], [True, False], [True, False]]
    if [len(g) for g in groups] != [len(e) for e in expect_relu]:
        raise NotPackable("unexpected layer counts")
    for g, e in zip(groups, expect_relu):
        if [r for _, _, r in g] != e:
            raise NotPackable("unexpected activation placement")
    layers = [(_fold(l, bn), relu) for g in groups for (l, bn, relu) in g]
    H = layers[0][0][0].shape[0]
    A = layers[0][0][0].shape[1] - H
    off = 4 if res else 2
    F = layers[off][0][0].shape[0]
    V = layers[off + 1][0][0].shape[0]
    if layers[-1][0][0].shape[0] != A:
        raise NotPackable("policy head width != action space")
    return layers, dict(hidden=H, actions=A, head_hidden=F, support=V, res=res)


def pack_muzero_mlp(model, device):
    layers, dims = describe(model)
    parts = []
    for (W, b), _ in layers:
        parts.append(W.t().contiguous().reshape(-1))
        parts.append(b.reshape(-1))
    flat = torch.cat(parts).to(device=device, dtype=torch.float32).contiguous()
    n = _lib.load().lzm_mlp_packed_floats(dims["hidden"], dims["actions"], dims["head_hidden"], dims["support"],
                                          int(dims["res"]))
    if n != flat.numel():
        raise NotPackable(f"packed size {flat.numel()} != expected {n}")
    return flat, dims


def prepare_kernel_weights(flat, dims, out=None):
    """Packed network -> the search kernel's lane-order layout (lzm_mlp_prepare, on the current stream);
    out: optional existing buffer of the right size to refill in place."""
    args = (dims["hidden"], dims["actions"], dims["head_hidden"], dims["support"], int(dims["res"]))
    n = _lib.load().lzm_mlp_kernel_floats(*args)
    if out is None or out.numel() != n or out.device != flat.device:
        out = torch.empty(n, dtype=torch.float32, device=flat.device)
    _lib.call("lzm_mlp_prepare", *args, _lib.ptr(flat), _lib.ptr(out), _lib.stream_ptr())
    return out


class PackedCache:
    """Kernel-layout weights per model (small LRU keyed by model identity and device). Re-packs only
    when the model's parameters or buffers change (tensor version counters), and then IN PLACE, so a
    HIP graph that captured a search over these weights keeps reading the current ones."""

    def __init__(self, cap=4):
        self.cap = int(cap)
        self._d = OrderedDict()  # (id(model), device) -> [model weakref, version, weights, dims]

    @staticmethod
    def _version(model):
        return tuple(t._version for t in list(model.parameters()) + list(model.buffers()))

    def get(self, model, device):
        key = (id(model), str(device))
        e = self._d.get(key)
        if e is not None and e[0]() is not model:  # a dead model's id was reused
            del self._d[key]
            e = None
        ver = self._version(model)
        if e is None:
            flat, dims = pack_muzero_mlp(model, device)
            e = [weakref.ref(model), ver, prepare_kernel_weights(flat, dims), dims]
            self._d[key] = e
            while len(self._d) > self.cap:
                self._d.popitem(last=False)
        elif e[1] != ver:
            flat, dims = pack_muzero_mlp(model, device)
            e[2] = prepare_kernel_weights(flat, dims, out=e[2] if dims == e[3] else None)
            e[1], e[3] = ver, dims
        self._d.move_to_end(key)
        return e[2], e[3]
