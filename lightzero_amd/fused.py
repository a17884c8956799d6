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


def prepare_kernel_weights(flat, dims):
    """Packed network -> the search kernel's lane-order layout (lzm_mlp_prepare, on the current stream)."""
    args = (dims["hidden"], dims["actions"], dims["head_hidden"], dims["support"], int(dims["res"]))
    n = _lib.load().lzm_mlp_kernel_floats(*args)
    out = torch.empty(n, dtype=torch.float32, device=flat.device)
    _lib.call("lzm_mlp_prepare", *args, _lib.ptr(flat), _lib.ptr(out), _lib.stream_ptr())
    return out


class PackedCache:
    """Kernel-layout weights of a model; re-packs only when the model's parameters or buffers
    change (tensor version counters)."""

    def __init__(self):
        self.key = None
        self.value = None

    def get(self, model, device):
        ver = tuple(t._version for t in list(model.parameters()) + list(model.buffers()))
        key = (id(model), str(device), ver)
        if key != self.key:
            flat, dims = pack_muzero_mlp(model, device)
            self.value = (prepare_kernel_weights(flat, dims), dims)
            self.key = key
        return self.value
