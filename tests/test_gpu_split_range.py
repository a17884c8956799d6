"""GPU: the split-fp16 paths (configs 3 and 5) outside the range of random-init weights — VERDICT r05 "What's
weak" 1 / ADVICE r05 medium 1.

The DownSample (csrc/lzm_repr.h), the recurrent conv trunk (csrc/lzm_conv.h) and the EfficientZero gate GEMM
(csrc/lzm_lstm.h) hold every f32 operand as two fp16 terms. Unscaled, fp16's range made |x| >= 65504 overflow
and cost the low term its precision below 2^-3; each path now scales weight rows and activation tensors by
powers of two (lzm_conv.h, "Range"). These tests drive the kernels with magnitudes the unscaled split could
not hold — activations ~1e5 and ~1e-5, weights ~1e-4 next to ~1e2 — and compare against float64 ELEMENT-WISE:

    |got - ref| <= tol * A,   A = the same network in float64 with every weight, bias and input replaced by its
                              absolute value and every ReLU by the identity,

A being the per-element scale an f32 evaluation's rounding error is proportional to (sum |w| |x| along every
path), so no element hides behind the tensor's largest one (tol = 2^-16), and the relative error |got - ref| /
|ref| of every element no worse than torch's own f32 evaluation of the same network shows (its median, 99th
percentile and max are printed beside ours).
A non-finite activation raises SplitRangeError from the searches' result getters (lzm_check_errors).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import bench

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)
TOL = 2.0 ** -16


def _rel(x, ref):
    """|x - ref| / |ref| over the elements with |ref| > 1e-6 max |ref| (the near-zeros a sum cancelled to excluded)"""
    nz = ref.abs() > 1e-6 * ref.abs().max()
    return (x - ref).abs()[nz] / ref.abs()[nz]


def _check(name, got, ref, A, f32):
    """element-wise against float64: |err| <= 2^-16 A everywhere, and the relative error |err| / |ref| no worse
    than an f32 evaluation of the same network (torch, CPU) shows: 99th percentile <= max(1e-5, 2x f32's),
    max <= max(1e-3, 4x f32's)"""
    got, ref, A, f32 = got.double().cpu(), ref.double().cpu(), A.double().cpu(), f32.double().cpu()
    ratio = float(((got - ref).abs() / A.clamp_min(1e-300)).max())
    rel, r32 = _rel(got, ref), _rel(f32, ref)
    q = [float(torch.quantile(rel, x)) for x in (0.5, 0.99, 1.0)]
    q32 = [float(torch.quantile(r32, x)) for x in (0.5, 0.99, 1.0)]
    print(f"{name}: max |err| / A = {ratio:.2e}; |err| / |ref| median / p99 / max: {q[0]:.2e} / {q[1]:.2e} / "
          f"{q[2]:.2e} (torch f32: {q32[0]:.2e} / {q32[1]:.2e} / {q32[2]:.2e}); max |ref| {float(ref.abs().max()):.2e}")
    assert torch.isfinite(got).all(), name
    assert ratio <= TOL, (name, ratio)
    assert q[1] <= max(1e-5, 2 * q32[1]) and q[2] <= max(1e-3, 4 * q32[2]), (name, q, q32)
    return ratio


# ---- the DownSample -------------------------------------------------------------------------------------
def _downsample64(ops, x, absolute=False):
    """float64 DownSample over FoldedConvInitial ops (absolute: |w|, |b|, identity ReLU: the error scale A)"""
    f = (lambda t: t.abs()) if absolute else (lambda t: t)
    act = (lambda t: t) if absolute else (lambda t: t.relu())
    x = f(x)
    for op in ops:
        if op[0] == "conv_relu":
            x = act(F.conv2d(x, f(op[1]), f(op[2]), stride=op[3], padding=1))
        elif op[0] == "basic":
            y = act(F.conv2d(x, f(op[1]), f(op[2]), padding=1))
            x = act(F.conv2d(y, f(op[3]), f(op[4]), padding=1) + x)
        elif op[0] == "down":
            y = act(F.conv2d(x, f(op[1]), f(op[2]), stride=2, padding=1))
            x = act(F.conv2d(y, f(op[3]), f(op[4]), padding=1) + F.conv2d(x, f(op[5]), None, stride=2, padding=1))
        else:
            x = F.avg_pool2d(x, 3, 2, 1)
    return x


@pytest.mark.parametrize("case", ["large", "small", "weights"])
def test_downsample_scaled_elementwise_vs_float64(case):
    """lzm_repr_downsample with the observation and every bias scaled by 1e5 ("large": every activation ~1e5,
    past fp16's 65504) or 1e-5 ("small": ~1e-5, fp16 subnormals), or with the first block's weights x1e-3 and
    the next conv's x1e3 ("weights": rows of ~1e-4 next to ~1e2): element-wise within 2^-16 of A"""
    from lightzero_amd.conv_infer import FoldedConvInitial
    m = bench.build_conv_model(DEV, seed=3)
    fi = FoldedConvInitial(m)
    i0 = fi.tail[0]
    s = {"large": 1e5, "small": 1e-5, "weights": 1.0}[case]
    with torch.no_grad():
        for op in fi.ops[:i0]:
            if op[0] == "conv_relu":
                op[2].mul_(s)
            elif op[0] in ("basic", "down"):
                op[2].mul_(s)
                op[4].mul_(s)
        if case == "weights":
            basic = [op for op in fi.ops[:i0] if op[0] == "basic"]
            basic[0][1].mul_(1e-3)
            basic[0][3].mul_(1e3)
        fi._pack_native()
        B = 37
        obs = torch.rand(B, 4, 64, 64, device=DEV) * s
        got = fi._downsample_native(obs)
        torch.cuda.synchronize()
    ops = [tuple(t.cpu().double() if torch.is_tensor(t) else t for t in op) for op in fi.ops[:i0]]
    x = obs.cpu().double()
    ref, A = _downsample64(ops, x), _downsample64(ops, x, absolute=True)
    ops32 = [tuple(t.cpu() if torch.is_tensor(t) else t for t in op) for op in fi.ops[:i0]]
    f32 = _downsample64(ops32, obs.cpu())
    _check(f"downsample {case}", got, ref, A, f32)


# ---- the recurrent trunk --------------------------------------------------------------------------------
def _trunk64(t, lat, act, n_dres, n_pres, absolute=False, dtype=torch.float64):
    """float64 (or dtype) recurrent conv step on FoldedConvNet tensors: (next latent, reward planes, head planes)"""
    d = {k: v.detach().to(dtype).cpu() for k, v in t.items()}
    lat = lat.to(dtype)
    f = (lambda z: z.abs()) if absolute else (lambda z: z)
    relu = (lambda z: z) if absolute else (lambda z: z.relu())
    lat = f(lat)
    x = relu(F.conv2d(lat, f(d["dyn_w"]), None, padding=1) + f(d["dyn_actmap"])[act] + lat)

    def blocks(x, name, n):
        for i in range(n):
            y = relu(F.conv2d(x, f(d[f"{name}{i}_w1"]), f(d[f"{name}{i}_b1"]), padding=1))
            x = relu(F.conv2d(y, f(d[f"{name}{i}_w2"]), f(d[f"{name}{i}_b2"]), padding=1) + x)
        return x
    nxt = blocks(x, "dres", n_dres)
    r = relu(F.conv2d(nxt, f(d["rw_w"]), f(d["rw_b"])))
    p = blocks(nxt, "pres", n_pres)
    h = relu(F.conv2d(p, f(d["head_w"]), f(d["head_b"])))
    B = lat.shape[0]
    return nxt, r.reshape(B, -1), h.reshape(B, -1)


@pytest.mark.parametrize("kind", ["mz", "ez"])
@pytest.mark.parametrize("case", ["large", "small", "weights"])
def test_trunk_scaled_elementwise_vs_float64(kind, case):
    """lzm_conv_trunk_p (split) with the latent and every bias / the action map scaled by 1e5 ("large") or
    1e-5 ("small"), or the first dynamics block's convs scaled x1e-3 / x1e3 ("weights"): next latent, reward
    planes and head planes element-wise within 2^-16 of A; no range error counted"""
    from lightzero_amd.conv_infer import FoldedConvNet
    from lightzero_amd.model_conv import atari_efficientzero_model
    if kind == "mz":
        m = bench.build_conv_model(DEV, seed=4)
    else:
        torch.manual_seed(4)
        m = atari_efficientzero_model(last_linear_layer_init_zero=False)
        bench._random_bn(m, 5)
        m = m.to(DEV).eval()
    net = FoldedConvNet(m, precision="split")
    t = net.t
    s = {"large": 1e5, "small": 1e-5, "weights": 1.0}[case]
    with torch.no_grad():
        for k in list(t):
            if k == "dyn_actmap" or (k.endswith(("_b1", "_b2")) and k[:4] in ("dres", "pres")) or k in ("rw_b", "head_b"):
                t[k].mul_(s)
        if case == "weights":
            t["dres0_w1"].mul_(1e-3)
            t["dres0_w2"].mul_(1e3)
        net._pack_native()
        B = 45
        g = torch.Generator(device=DEV).manual_seed(7)
        lat = torch.relu(torch.randn(B, 64, 8, 8, generator=g, device=DEV)) * s
        act = torch.randint(0, m.action_space_size, (B,), generator=g, device=DEV).to(torch.int32)
        out = torch.empty(B, 64, 8, 8, device=DEV)
        err = torch.zeros(1, dtype=torch.int32, device=DEV)
        from lightzero_amd import _lib
        r, h = net._trunk(lat.unsqueeze(0).contiguous(), torch.zeros(B, dtype=torch.int32, device=DEV), act, out,
                          _lib.ptr(err))
        torch.cuda.synchronize()
    assert int(err.item()) == 0
    a = act.long().cpu()
    ref = _trunk64(t, lat.cpu().double(), a, net.n_dres, net.n_pres)
    A = _trunk64(t, lat.cpu().double(), a, net.n_dres, net.n_pres, absolute=True)
    f32 = _trunk64(t, lat.cpu(), a, net.n_dres, net.n_pres, dtype=torch.float32)
    for name, x, y, z, w in zip(("latent", "reward planes", "head planes"), (out, r, h), ref, A, f32):
        _check(f"trunk {kind} {case} {name}", x.reshape(y.shape), y, z, w)


# ---- the EfficientZero gate GEMM --------------------------------------------------------------------------
@pytest.mark.parametrize("case", ["large", "small"])
def test_lstm_gate_gemm_scaled_elementwise_vs_float64(case):
    """lzm_ez_lstm_step (split-fp16 gate GEMM + cell) with the reward-plane part of xin scaled by 1e5 and its
    gate weights by 1e-5 ("large": inputs past fp16's range, weights in its subnormals) or the reverse
    ("small"), the hidden-state part at its natural scale, rows of different magnitude (1 .. 1e3 per row):
    the new h / c element-wise within 2^-16 of the gates' A (sum |w| |x| + |b|, max over the unit's gates,
    times (1 + |c0|)), against float64"""
    from lightzero_amd import _lib
    B, Kr, H = 70, 1024, 512
    K = Kr + H
    s = {"large": 1e5, "small": 1e-5}[case]
    g = torch.Generator().manual_seed(11)
    rowmag = torch.logspace(0, 3, B, dtype=torch.float64).unsqueeze(1)
    xr = torch.relu(torch.randn(B, Kr, generator=g, dtype=torch.float64)) * s / rowmag
    xh = torch.tanh(torch.randn(B, H, generator=g, dtype=torch.float64))
    xin64 = torch.cat([xr, xh], dim=1).float().double()
    W64 = (torch.randn(4 * H, K, generator=g, dtype=torch.float64) * 0.03)
    W64[:, :Kr] /= s
    W64 = W64.float().double()
    b64 = (torch.randn(4 * H, generator=g, dtype=torch.float64) * 0.1).float().double()
    c0 = (torch.randn(B, H, generator=g, dtype=torch.float64) * 0.5).float().double()
    L = _lib.load()
    nfl = L.lzm_ez_lstm_frag_floats(K, H)
    host = np.zeros(nfl, np.float32)
    Wn = np.ascontiguousarray(W64.float().numpy())
    _lib.check(L.lzm_ez_lstm_prepare(K, H, Wn.ctypes.data, host.ctypes.data), "prepare")
    frag = torch.from_numpy(host).to(DEV)
    xin = xin64.float().to(DEV).contiguous()
    bias = b64.float().to(DEV)
    cpool = c0.float().to(DEV).unsqueeze(0).contiguous()
    x = torch.zeros(B, dtype=torch.int32, device=DEV)
    slen = torch.ones(B, dtype=torch.int32, device=DEV)
    outs = [torch.empty(B, H, device=DEV) for _ in range(4)]
    ws = torch.zeros((int(L.lzm_ez_lstm_workspace_bytes(B, H)) + 15) // 16 * 4, device=DEV)
    werr = torch.zeros(2, dtype=torch.int32, device=DEV)
    # the rows' scale exponents as the trunk computes them (lzm_conv.h ls_row_exp: the reward planes' max, >= 1)
    rmax = xr.float().abs().amax(dim=1).double().clamp_min(1.0)
    xscale = (14 - torch.floor(torch.log2(rmax))).to(torch.int32).to(DEV)
    P = _lib.ptr
    _lib.call("lzm_ez_lstm_step", B, K, H, P(xin), P(xscale), P(frag), P(bias), P(cpool), P(x), P(slen), 5,
              P(outs[0]), P(outs[1]), P(outs[2]), P(outs[3]), P(ws), P(werr), P(werr[1:]), _lib.stream_ptr())
    torch.cuda.synchronize()
    assert werr.tolist() == [0, 0]
    def cell(x, W, b, c):
        gi, gf, gg, go = (x @ W.t() + b).chunk(4, dim=1)
        c1 = torch.sigmoid(gf) * c + torch.sigmoid(gi) * torch.tanh(gg)
        return torch.sigmoid(go) * torch.tanh(c1), c1
    h1, c1 = cell(xin64, W64, b64, c0)
    h32, c32 = cell(xin64.float(), W64.float(), b64.float(), c0.float())
    Ag = xin64.abs() @ W64.abs().t() + b64.abs()
    A = torch.stack(Ag.chunk(4, dim=1)).amax(dim=0) * (1 + c0.abs())
    _check(f"lstm {case} h1", outs[0], h1, A, h32)
    _check(f"lstm {case} c1", outs[1], c1, A, c32)


# ---- non-finite values: the range error -------------------------------------------------------------------
@pytest.mark.parametrize("kind", ["mz", "ez"])
@pytest.mark.parametrize("fused", [True, False])
def test_nonfinite_latent_raises_split_range_error(kind, fused):
    """a NaN in one root's latent: the search's split trunk counts it (error word 4) and the first result getter
    raises SplitRangeError (one-launch and generic paths); the next search on the same tree is clean"""
    from lightzero_amd import _lib
    from lightzero_amd.mcts_ctree import EfficientZeroMCTSCtree, MuZeroMCTSCtree
    from lightzero_amd.utils import EasyDict
    from tests.test_gpu_conv import conv_model
    model = conv_model(kind, 5)
    B, S = 16, 6
    A = model.action_space_size
    obs = torch.rand(B, 4, 64, 64, device=DEV)
    with torch.no_grad():
        out = model.initial_inference(obs)
    cls = EfficientZeroMCTSCtree if kind == "ez" else MuZeroMCTSCtree
    cfg = EasyDict(dict(num_simulations=S, discount_factor=0.997, device=DEV, lstm_horizon_len=5, fused_search=fused,
                        model=dict(support_scale=50 if kind == "ez" else 300, categorical_distribution=True)))
    mcts = cls(cfg)
    logits = out.policy_logits.float().cpu().tolist()
    for bad in (True, False):
        lat = out.latent_state.clone()
        if bad:
            lat[3, 5, 2, 2] = float("nan")
        roots = cls.roots(B, [list(range(A))] * B)
        roots.prepare_no_noise([0.0] * B, logits, [-1] * B)
        if kind == "ez":
            mcts.search(roots, model, lat, out.reward_hidden_state, [-1] * B)
        else:
            mcts.search(roots, model, lat, [-1] * B)
        if bad:
            with pytest.raises(_lib.SplitRangeError):
                roots.get_distributions()
        else:
            assert np.array(roots.get_distributions()).sum() == B * S
        roots.clear()


# ---- network in the loop: configs 3 and 5 ----------------------------------------------------------------
@pytest.mark.parametrize("kind", ["mz", "ez"])
def test_fused_vs_torch_module_search_divergence_conv(kind):
    """Configs 5 (Breakout MuZero) / 3 (Pong EfficientZero) at 256 x 50: the one-launch search (split-fp16
    network inside the kernel) against the generic path with the torch module itself in the loop (no
    folding, MIOpen / rocBLAS f32), same roots, seeds and weights. Each tree reproduces the oracle fed its own
    network outputs; every root's first divergent walk is a pUCT near-tie moved by rounding or a glibc draw
    taken at a shifted stream position after an earlier root diverged (tests/divergence.py). Reported to
    $LZM_REPORT_DIR/divergence_conv_<kind>_fused_vs_torch.json (DESIGN.md §3 quotes it)."""
    from lightzero_amd.mcts_ctree import EfficientZeroMCTSCtree, MuZeroMCTSCtree
    from lightzero_amd.utils import EasyDict
    from tests.divergence import attribute, report
    from tests.test_gpu_conv import conv_model, run_search
    B, S = 256, 50
    model = conv_model(kind, 11)
    cls = EfficientZeroMCTSCtree if kind == "ez" else MuZeroMCTSCtree
    res = {}
    for name, fused in (("fused", True), ("torch", False)):
        cfg = EasyDict(dict(num_simulations=S, discount_factor=0.997, device=DEV, lstm_horizon_len=5,
                            fused_search=fused, fold_network=fused,
                            model=dict(support_scale=50 if kind == "ez" else 300, categorical_distribution=True)))
        res[name] = run_search(kind, B, S, seed=12, model=model, mcts=cls(cfg))
    assert res["fused"]["path"] in ("fused", "fused-conv") and res["torch"]["path"] == "generic"
    rep = attribute(res["fused"], res["torch"], B, S, res["fused"]["A"], ez=(kind == "ez"), tau=1e-3)
    report(f"conv_{kind}_fused_vs_torch", rep)
    kinds = rep["first_divergence_kinds"]
    assert kinds.get("unexplained", 0) == 0, rep["first_divergences"][:5]
    assert kinds.get("tie_draw", 0) == 0
    assert rep["rate"] <= 0.1, rep["rate"]
