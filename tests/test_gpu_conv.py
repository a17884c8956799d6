"""GPU: the convolutional Atari configs through the drop-in search (BASELINE.json configs 3 and 5).

Config 3 — Pong EfficientZero: EfficientZeroMCTSCtree.search with the restated EfficientZeroModel
(latent 64x8x8, LSTM 512, support 101, 6 actions, lstm_horizon_len 5).
Config 5 — Breakout MuZero: MuZeroMCTSCtree.search with the restated MuZeroModel (latent 64x8x8,
support 601, 4 actions); the 8-GPU sharding itself is covered by tests/test_dist.py.

Parity as for the other categorical searches (tests/test_gpu_search.py): the tree, fed the decoded
values it consumed, equals the oracle bit for bit (requests at every simulation, visit counts,
root values, trajectories; EZ also is_reset), and the decoded values equal a torch fp32
InverseScalarTransform of the same network outputs within rtol 1e-4 / atol 1e-5 x support_scale.
The network is the model's own PyTorch-ROCm forward (not pinned to the reference: DI-engine absent).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from oracle.oracle import OracleTree  # noqa: E402
from tests.helpers import DISC, NOISE_W, PB_C_BASE, PB_C_INIT, VDM  # noqa: E402
from tests.test_gpu_numerics import torch_inverse_scalar_transform  # noqa: E402

DEV = torch.device("cuda", 0)


def conv_model(kind, seed=0, zero_heads=False):
    from lightzero_amd.model_conv import atari_efficientzero_model, atari_muzero_model
    torch.manual_seed(seed)
    m = (atari_efficientzero_model if kind == "ez" else atari_muzero_model)(last_linear_layer_init_zero=zero_heads)
    g = torch.Generator().manual_seed(seed + 1)
    for mod in m.modules():  # non-trivial eval-mode BatchNorm statistics
        if isinstance(mod, (torch.nn.BatchNorm1d, torch.nn.BatchNorm2d)):
            n = mod.num_features
            mod.running_mean.copy_(torch.randn(n, generator=g) * 0.1)
            mod.running_var.copy_(torch.rand(n, generator=g) + 0.5)
            mod.weight.data.copy_(torch.rand(n, generator=g) + 0.5)
            mod.bias.data.copy_(torch.randn(n, generator=g) * 0.1)
    return m.to(DEV).eval()


def run_search(kind, B, S, seed, graph=False, record=True, model=None, mcts=None, fused=True, rng="glibc"):
    from lightzero_amd.mcts_ctree import EfficientZeroMCTSCtree, MuZeroMCTSCtree
    from lightzero_amd.tree import SequentialSeeds, set_seed_source
    from lightzero_amd.utils import EasyDict
    model = conv_model(kind, seed) if model is None else model
    A = model.action_space_size
    scale = 50 if kind == "ez" else 300
    rng = np.random.default_rng(seed)
    obs = torch.from_numpy(rng.integers(0, 256, size=(B, 4, 64, 64)).astype(np.float32) / 255.0).to(DEV)
    with torch.no_grad():
        out = model.initial_inference(obs)
    noises = rng.dirichlet([0.3] * A, size=B).astype(np.float32)
    logits0 = out.policy_logits.float().cpu().numpy()
    cfg = EasyDict(dict(num_simulations=S, discount_factor=0.997, device=DEV, lstm_horizon_len=5,
                        use_hip_graph=graph, fused_search=fused,
                        model=dict(support_scale=scale, categorical_distribution=True)))
    cls = EfficientZeroMCTSCtree if kind == "ez" else MuZeroMCTSCtree
    mcts = cls(cfg) if mcts is None else mcts
    mcts.record = record
    old_mode = cls.rng_mode
    cls.rng_mode = rng
    try:
        roots = cls.roots(B, [list(range(A))] * B)
    finally:
        cls.rng_mode = old_mode
    roots.prepare(0.25, [n.tolist() for n in noises], [0.0] * B, logits0.tolist(), [-1] * B)
    set_seed_source(SequentialSeeds(seed))
    try:
        if kind == "ez":
            mcts.search(roots, model, out.latent_state, out.reward_hidden_state, [-1] * B)
        else:
            mcts.search(roots, model, out.latent_state, [-1] * B)
    finally:
        set_seed_source(None)
    t = roots.tree
    res = dict(dist=t.distributions().cpu().numpy(), values=t.values().cpu().numpy(),
               traj=t.trajectories(S + 2).cpu().numpy(), noises=noises, logits0=logits0, model=model,
               lat0=out.latent_state, hidden0=getattr(out, "reward_hidden_state", None), A=A, scale=scale)
    res["rec"] = None if mcts.last_record is None else mcts.last_record.numpy() | (
        {"is_reset": mcts.last_record.is_reset.cpu().numpy()} if kind == "ez" else {})
    res["path"] = getattr(mcts, "last_path", None)
    roots.clear()
    return res


def oracle_replay(kind, res, B, S):
    rec, A = res["rec"], res["A"]
    ot = OracleTree(B, A, S, ez=(kind == "ez"))
    ot.set_delta(VDM)
    ot.prepare(NOISE_W, res["noises"], np.zeros(B, np.float32), res["logits0"], np.full(B, -1, np.int32))
    for k in range(S):
        x, y, a, vtp, slen = ot.traverse(PB_C_BASE, PB_C_INIT, DISC, int(rec["seeds"][k]), np.full(B, -1, np.int32))
        assert np.array_equal(x, rec["x"][k]), f"sim {k}: latent index differs"
        assert np.array_equal(a, rec["action"][k]), f"sim {k}: action differs"
        assert np.array_equal(slen, rec["search_len"][k]), f"sim {k}: search_len differs"
        is_reset = None
        if kind == "ez":
            is_reset = (slen % 5 == 0).astype(np.int32)
            assert np.array_equal(is_reset, rec["is_reset"][k]), f"sim {k}: is_reset differs"
        ot.backprop(k + 1, DISC, rec["decoded"][k][:, 0], rec["decoded"][k][:, 1], rec["policy_logits"][k], vtp,
                    is_reset)
    assert np.array_equal(res["dist"], ot.distributions())
    assert np.array_equal(res["values"], ot.values())
    assert np.array_equal(res["traj"], ot.trajectories(S + 2))


def torch_replay(kind, res, B, S):
    """the decoded values the kernel consumed == torch InverseScalarTransform of the same net outputs"""
    rec, model, scale = res["rec"], res["model"], res["scale"]
    pool = [res["lat0"].float()]
    if kind == "ez":
        hpool = [(res["hidden0"][0].reshape(B, -1).float(), res["hidden0"][1].reshape(B, -1).float())]
    rows = torch.arange(B, device=DEV)
    with torch.no_grad():
        for k in range(S):
            xs = torch.from_numpy(rec["x"][k]).long().to(DEV)
            lat = torch.stack(pool)[xs, rows]
            act = torch.from_numpy(rec["action"][k]).long().to(DEV)
            if kind == "ez":
                hs = torch.stack([h[0] for h in hpool])[xs, rows], torch.stack([h[1] for h in hpool])[xs, rows]
                out = model.recurrent_inference(lat, (hs[0].unsqueeze(0), hs[1].unsqueeze(0)), act)
                r_logits = out.value_prefix
                keep = torch.from_numpy(1 - rec["is_reset"][k]).float().to(DEV).unsqueeze(1)
                hc, hh = out.reward_hidden_state
                hpool.append((hc.reshape(B, -1) * keep, hh.reshape(B, -1) * keep))
            else:
                out = model.recurrent_inference(lat, act)
                r_logits = out.reward
            dec = torch.from_numpy(rec["decoded"][k]).to(DEV)
            torch.testing.assert_close(dec[:, 0], torch_inverse_scalar_transform(r_logits, scale).squeeze(1),
                                       rtol=1e-4, atol=1e-5 * scale)
            torch.testing.assert_close(dec[:, 1], torch_inverse_scalar_transform(out.value, scale).squeeze(1),
                                       rtol=1e-4, atol=1e-5 * scale)
            torch.testing.assert_close(torch.from_numpy(rec["policy_logits"][k]).to(DEV), out.policy_logits.float(),
                                       rtol=1e-4, atol=1e-5)
            pool.append(out.latent_state.float())


@pytest.mark.parametrize("kind,B,S", [("ez", 16, 12), ("mz", 16, 12)])
def test_conv_search_tree_and_decode_parity(kind, B, S):
    res = run_search(kind, B, S, seed=1)
    oracle_replay(kind, res, B, S)
    torch_replay(kind, res, B, S)


@pytest.mark.parametrize("kind,fused", [("ez", True), ("ez", False), ("mz", True), ("mz", False)])
def test_conv_search_full_config_tree_parity(kind, fused):
    """configs 3 / 5 at their per-GPU size: 256 envs x 50 simulations (the one-launch searches,
    lzm_search_conv / lzm_search_conv_ez, and the generic per-simulation path)"""
    B, S = 256, 50
    res = run_search(kind, B, S, seed=2, fused=fused)
    oracle_replay(kind, res, B, S)
    assert (res["dist"].sum(axis=1) == S).all()


@pytest.mark.parametrize("kind", ["mz", "ez"])
@pytest.mark.parametrize("B,S,rng,zero", [(256, 50, "glibc", False), (64, 30, "glibc", True), (37, 20, "philox", False)])
def test_fused_conv_search_equals_generic(kind, B, S, rng, zero):
    """lzm_search_conv / lzm_search_conv_ez (one launch for all simulations) run the generic path's
    arithmetic in the same order: identical requests at every simulation, decoded values, policy
    logits, visit counts, root values and trajectories (EZ: is_reset too), in both RNG modes; with
    zero-init heads (all-tie search: ties reaching expanded children take the serial draw path) too.
    EZ at B = 37: 64 workgroups, 27 of them LSTM tiles without a root."""
    model = conv_model(kind, 13, zero_heads=zero)
    out = [run_search(kind, B, S, seed=14, model=model, fused=f, rng=rng) for f in (True, False)]
    a, b = out
    # the one-launch search really ran (EZ: the co-residency bound accepted the grid)
    assert a["path"] in ("fused", "fused-conv") and b["path"] == "generic", (a["path"], b["path"])
    for key in ("dist", "values", "traj"):
        assert np.array_equal(a[key], b[key]), key
    for key in ("x", "action", "search_len", "decoded", "policy_logits") + (("is_reset",) if kind == "ez" else ()):
        assert np.array_equal(a["rec"][key], b["rec"][key]), key
    if rng == "glibc":
        oracle_replay(kind, a, B, S)


def test_fused_conv_search_beyond_cu_count():
    """the one-launch MuZero conv search with more roots than CUs (600: the workgroups past the CU count queue
    behind the first ones, and each look-back sums three 256-root chunks) — the fused path runs and equals the
    generic path and the oracle bit for bit"""
    B, S = 600, 20
    model = conv_model("mz", 15)
    a, b = [run_search("mz", B, S, seed=16, model=model, fused=f) for f in (True, False)]
    assert a["path"] in ("fused", "fused-conv") and b["path"] == "generic", (a["path"], b["path"])
    for key in ("dist", "values", "traj"):
        assert np.array_equal(a[key], b[key]), key
    for key in ("x", "action", "search_len", "decoded", "policy_logits"):
        assert np.array_equal(a["rec"][key], b["rec"][key]), key
    oracle_replay("mz", a, B, S)


def test_fused_conv_search_head_weight_copy_on_off(monkeypatch):
    """the Breakout search's LDS copy of the first head half-head (default on when every root has a CU) against
    LZM_CONV_PIN=0 (every head weight from L2): the same bits, and both equal the oracle"""
    B, S = 256, 20
    model = conv_model("mz", 17)
    runs = []
    for pin in ("1", "0"):
        monkeypatch.setenv("LZM_CONV_PIN", pin)
        runs.append(run_search("mz", B, S, seed=18, model=model, fused=True))
    a, b = runs
    assert a["path"] in ("fused", "fused-conv") and b["path"] == a["path"], (a["path"], b["path"])
    for key in ("dist", "values", "traj"):
        assert np.array_equal(a[key], b[key]), key
    for key in ("x", "action", "search_len", "decoded", "policy_logits"):
        assert np.array_equal(a["rec"][key], b["rec"][key]), key
    oracle_replay("mz", a, B, S)


def test_fused_ez_search_pools_equal_generic():
    """the one-launch EZ search files the same latent and LSTM state pools as the generic path
    (next latents, reset-masked h / c slots, mcts_ctree.py:805-816)"""
    from lightzero_amd.mcts_ctree import EfficientZeroMCTSCtree
    from lightzero_amd.utils import EasyDict
    model = conv_model("ez", 21)
    B, S = 64, 12
    bufs = []
    for f in (True, False):
        cfg = EasyDict(dict(num_simulations=S, discount_factor=0.997, device=DEV, lstm_horizon_len=5,
                            use_hip_graph=False, fused_search=f,
                            model=dict(support_scale=50, categorical_distribution=True)))
        mcts = EfficientZeroMCTSCtree(cfg)
        run_search("ez", B, S, seed=22, model=model, mcts=mcts)
        bufs.append([x.clone() for x in (mcts._buf.pool, mcts._buf.extra[0], mcts._buf.extra[1])])
    for name, x, y in zip(("latent", "h", "c"), *bufs):
        assert torch.equal(x, y), name


@pytest.mark.parametrize("kind", ["ez", "mz"])
def test_conv_search_graph_replay_equals_eager(kind):
    B, S = 64, 20
    model = conv_model(kind, 3)
    from lightzero_amd.mcts_ctree import EfficientZeroMCTSCtree, MuZeroMCTSCtree
    from lightzero_amd.utils import EasyDict
    eager = run_search(kind, B, S, seed=3, model=model, record=False, fused=False)
    cls = EfficientZeroMCTSCtree if kind == "ez" else MuZeroMCTSCtree
    cfg = EasyDict(dict(num_simulations=S, discount_factor=0.997, device=DEV, lstm_horizon_len=5, use_hip_graph=True,
                        fused_search=False,
                        model=dict(support_scale=50 if kind == "ez" else 300, categorical_distribution=True)))
    mcts = cls(cfg)
    for _ in range(2):  # capture, then a plain replay of the cached graph
        graph = run_search(kind, B, S, seed=3, model=model, record=False, mcts=mcts, fused=False)
        assert np.array_equal(graph["dist"], eager["dist"])
        np.testing.assert_allclose(graph["values"], eager["values"], rtol=0, atol=1e-6)


@pytest.mark.parametrize("precision", ["bf16x3", "f32"])
@pytest.mark.parametrize("kind", ["ez", "mz"])
def test_native_trunk_matches_module(kind, precision):
    """lzm_conv_trunk_p (+ batched heads) == the module's recurrent_inference (fp32, rtol 1e-4 / atol 1e-5),
    for the split-bf16 trunk (the default) and the exact-f32 one"""
    from lightzero_amd.conv_infer import FoldedConvNet
    model = conv_model(kind, 5)
    net = FoldedConvNet(model, precision=precision)
    assert net.native is not None, "native trunk not packed on the GPU"
    B = 37
    g = torch.Generator(device=DEV).manual_seed(0)
    lat = torch.relu(torch.randn(B, 64, 8, 8, generator=g, device=DEV))
    act = torch.randint(0, model.action_space_size, (B,), generator=g, device=DEV)
    with torch.no_grad():
        if kind == "ez":
            hc = (torch.randn(1, B, 512, generator=g, device=DEV) * 0.5, torch.randn(1, B, 512, generator=g, device=DEV) * 0.5)
            ref, got = model.recurrent_inference(lat, hc, act), net.recurrent_inference(lat, hc, act)
            torch.testing.assert_close(got.value_prefix, ref.value_prefix, rtol=1e-4, atol=1e-5)
            for a, b in zip(got.reward_hidden_state, ref.reward_hidden_state):
                torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5)
        else:
            ref, got = model.recurrent_inference(lat, act), net.recurrent_inference(lat, act)
            torch.testing.assert_close(got.reward, ref.reward, rtol=1e-4, atol=1e-5)
        torch.testing.assert_close(got.latent_state, ref.latent_state, rtol=1e-4, atol=1e-5)
        torch.testing.assert_close(got.value, ref.value, rtol=1e-4, atol=1e-5)
        torch.testing.assert_close(got.policy_logits, ref.policy_logits, rtol=1e-4, atol=1e-5)
        # pool-indexed form: leaf latents pool[x[b]][b], next latent into a pool slot
        pool = torch.relu(torch.randn(4, B, 64, 8, 8, generator=g, device=DEV))
        x = torch.randint(0, 4, (B,), generator=g, device=DEV).to(torch.int32)
        slot = torch.empty(B, 64, 8, 8, device=DEV)
        hid = hc if kind == "ez" else None
        o1 = net.step_from_pool(pool, x, act.to(torch.int32), slot, hid)
        leaf = pool[x.long(), torch.arange(B, device=DEV)]
        o2 = net.recurrent_inference(leaf, hc, act) if kind == "ez" else net.recurrent_inference(leaf, act)
        assert torch.equal(slot, o2.latent_state) and torch.equal(o1.value, o2.value)
        assert torch.equal(o1.policy_logits, o2.policy_logits)


def test_native_lstm_step_matches_module():
    """EZ on the pools: trunk + lzm_ez_lstm_input / rocBLAS gates / lzm_ez_lstm_cell + heads == the
    module's recurrent_inference on the gathered inputs (fp32, rtol 1e-4 / atol 1e-5), and the next
    state slots hold the new state zeroed where search_len % horizon == 0 (mcts_ctree.py:810-813)."""
    from lightzero_amd.conv_infer import FoldedConvNet
    model = conv_model("ez", 6)
    net = FoldedConvNet(model)
    assert net.native is not None, "native trunk not packed on the GPU"
    B, slots, H = 37, 4, 512
    g = torch.Generator(device=DEV).manual_seed(2)
    pool = torch.relu(torch.randn(slots, B, 64, 8, 8, generator=g, device=DEV))
    hpool = torch.randn(slots + 1, B, H, generator=g, device=DEV) * 0.5
    cpool = torch.randn(slots + 1, B, H, generator=g, device=DEV) * 0.5
    x = torch.randint(0, slots, (B,), generator=g, device=DEV).to(torch.int32)
    act = torch.randint(0, model.action_space_size, (B,), generator=g, device=DEV)
    slen = torch.randint(1, 13, (B,), generator=g, device=DEV).to(torch.int32)
    rows = torch.arange(B, device=DEV)
    xl = x.long()
    with torch.no_grad():
        ref = model.recurrent_inference(pool[xl, rows], (hpool[xl, rows].unsqueeze(0), cpool[xl, rows].unsqueeze(0)),
                                        act)
        slot = torch.empty(B, 64, 8, 8, device=DEV)
        got = net.step_from_pool_lstm(pool, x, act.to(torch.int32), slot, hpool, cpool, slots - 1, slen, 5)
    for name in ("value_prefix", "value", "policy_logits"):
        torch.testing.assert_close(getattr(got, name), getattr(ref, name), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(slot, ref.latent_state, rtol=1e-4, atol=1e-5)
    keep = (slen % 5 != 0).float().unsqueeze(1)
    h1, c1 = (s.reshape(B, H) for s in ref.reward_hidden_state)
    torch.testing.assert_close(hpool[slots], h1 * keep, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(cpool[slots], c1 * keep, rtol=1e-4, atol=1e-5)
    assert torch.all(hpool[slots][slen % 5 == 0] == 0) and torch.all(cpool[slots][slen % 5 == 0] == 0)


@pytest.mark.parametrize("B", [37, 256])
def test_fused_lstm_gate_gemm_cell_close_to_f32_gemm(B):
    """lzm_ez_lstm_step (gate GEMM on split-bf16 MFMA + cell in the epilogue, one launch) vs the f32
    rocBLAS GEMM + lzm_ez_lstm_cell on the same inputs: new state slots and head outputs within
    rtol 1e-4 / atol 1e-5 (both are f32-level: K = 1536 products summed in different orders differ by
    a few 1e-6 absolute; a plain bf16 GEMM would miss by ~1e-2), reset masks identical"""
    from lightzero_amd.conv_infer import FoldedConvNet
    model = conv_model("ez", 6)
    net = FoldedConvNet(model)
    assert net.lstm_frag is not None and net.lstm_fused, "fused LSTM step not packed"
    slots, H = 4, 512
    g = torch.Generator(device=DEV).manual_seed(5)
    pool = torch.relu(torch.randn(slots, B, 64, 8, 8, generator=g, device=DEV))
    hpool0 = torch.randn(slots + 1, B, H, generator=g, device=DEV) * 0.5
    cpool0 = torch.randn(slots + 1, B, H, generator=g, device=DEV) * 0.5
    x = torch.randint(0, slots, (B,), generator=g, device=DEV).to(torch.int32)
    act = torch.randint(0, model.action_space_size, (B,), generator=g, device=DEV).to(torch.int32)
    slen = torch.randint(1, 13, (B,), generator=g, device=DEV).to(torch.int32)
    res = []
    for fused in (True, False):
        net.lstm_fused = fused
        hpool, cpool = hpool0.clone(), cpool0.clone()
        slot = torch.empty(B, 64, 8, 8, device=DEV)
        with torch.no_grad():
            out = net.step_from_pool_lstm(pool, x, act, slot, hpool, cpool, slots - 1, slen, 5)
        torch.cuda.synchronize()
        res.append((out, hpool[slots].clone(), cpool[slots].clone()))
    net.lstm_fused = True
    (o1, h1, c1), (o0, h0, c0) = res
    torch.testing.assert_close(h1, h0, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(c1, c0, rtol=1e-4, atol=1e-5)
    assert torch.equal(h1 == 0, h0 == 0) and torch.all(h1[slen % 5 == 0] == 0)
    for name in ("value_prefix", "value", "policy_logits"):
        torch.testing.assert_close(getattr(o1, name), getattr(o0, name), rtol=1e-4, atol=1e-5)
    assert net.lstm_errors() == 0


@pytest.mark.parametrize("kind", ["ez", "mz"])
def test_fused_decode_traverse_equals_separate(kind):
    """cfg.fuse_traverse (lzm_decode_backprop_traverse: backup of simulation k and traverse of k + 1 in
    one launch) gives the same search as the two launches: requests, visit counts, values, trajectories"""
    from lightzero_amd.mcts_ctree import EfficientZeroMCTSCtree, MuZeroMCTSCtree
    from lightzero_amd.utils import EasyDict
    B, S = 64, 12
    model = conv_model(kind, 4)
    cls = EfficientZeroMCTSCtree if kind == "ez" else MuZeroMCTSCtree
    out = []
    for fuse in (False, True):
        cfg = EasyDict(dict(num_simulations=S, discount_factor=0.997, device=DEV, lstm_horizon_len=5,
                            fuse_traverse=fuse, fused_search=False,
                            model=dict(support_scale=50 if kind == "ez" else 300, categorical_distribution=True)))
        out.append(run_search(kind, B, S, seed=5, model=model, mcts=cls(cfg)))
    a, b = out
    for key in ("dist", "values", "traj"):
        assert np.array_equal(a[key], b[key]), key
    for key in ("x", "action", "search_len"):
        assert np.array_equal(a["rec"][key], b["rec"][key]), key


@pytest.mark.parametrize("B", [37, 256])
def test_heads_kernel_verdict_words(B):
    """lzm_conv_heads(norm_words): word pair q / head h is 1 iff every reward (h = 0) / value (h = 1)
    row of env block q sums to 1 within allclose(1e-5, 1e-5) (ensure_softmax,
    scaling_transform.py:36-62); pairs past the blocks are 1. Checked with output layers that
    give exactly normalised rows (zero weights, bias 1/V) and with random ones."""
    from lightzero_amd import _lib
    g = torch.Generator(device=DEV).manual_seed(3)
    Kr, Khd, fv, Vr, Vv, A = 1024, 2048, 1024, 601, 601, 4
    r = torch.rand(B, Kr, generator=g, device=DEV)
    hd = torch.rand(B, Khd, generator=g, device=DEV)
    w1t = torch.randn(3, 8, 32, 32, 4, generator=g, device=DEV) * 0.01
    b1 = torch.randn(96, generator=g, device=DEV) * 0.1
    nparts = (B + 1) // 2
    P = _lib.ptr
    for normalised in (True, False):
        if normalised:
            w2t = torch.zeros(32, Vr + Vv + A, device=DEV)
            b2 = torch.cat([torch.full((Vr,), 1.0 / Vr), torch.full((Vv,), 1.0 / Vv), torch.zeros(A)]).to(DEV)
        else:
            w2t = torch.randn(32, Vr + Vv + A, generator=g, device=DEV)
            b2 = torch.randn(Vr + Vv + A, generator=g, device=DEV)
        outs = [torch.empty(B, n, device=DEV) for n in (Vr, Vv, A)]
        words = torch.full((2 * nparts,), -7, dtype=torch.int32, device=DEV)
        _lib.call("lzm_conv_heads", B, Kr, Khd, fv, P(r), None, None, P(hd), P(w1t), P(b1), P(w2t), P(b2), Vr, Vv, A,
                  P(outs[0]), P(outs[1]), P(outs[2]), P(words), _lib.stream_ptr())
        torch.cuda.synchronize()
        w = words.cpu().numpy().reshape(nparts, 2)
        sums = [outs[h].sum(dim=1).cpu().numpy() for h in (0, 1)]
        nb = (B + 1) // 2  # env blocks of 2
        for h in (0, 1):
            ok = np.abs(sums[h] - 1.0) <= 2e-5
            exp = np.ones(nparts, np.int32)
            for q in range(nb):
                exp[q] = int(ok[2 * q:2 * q + 2].all())
            assert np.array_equal(w[:, h], exp), (normalised, h)
        assert w.all() == normalised


@pytest.mark.parametrize("kind", ["ez", "mz"])
def test_split_bf16_trunk_close_to_exact_f32(kind):
    """the split-bf16 trunk (six bf16 products per K) against the exact-f32 MFMA trunk on the same
    folded weights: next latents and head planes agree to f32 round-off (rtol 2e-5 / atol 2e-6), and
    the reported worst relative gap is far below the module tolerance"""
    from lightzero_amd.conv_infer import FoldedConvNet
    model = conv_model(kind, 9)
    nets = {p: FoldedConvNet(model, precision=p) for p in ("f32", "bf16x3")}
    B = 64
    g = torch.Generator(device=DEV).manual_seed(4)
    pool = torch.relu(torch.randn(3, B, 64, 8, 8, generator=g, device=DEV))
    x = torch.randint(0, 3, (B,), generator=g, device=DEV).to(torch.int32)
    act = torch.randint(0, model.action_space_size, (B,), generator=g, device=DEV).to(torch.int32)
    outs = {}
    for p, net in nets.items():
        lat = torch.empty(B, 64, 8, 8, device=DEV)
        r, h = net._trunk(pool, x, act, lat)
        outs[p] = (lat, r, h)
    for a, b in zip(outs["bf16x3"], outs["f32"]):
        torch.testing.assert_close(a, b, rtol=2e-5, atol=2e-6)


@pytest.mark.parametrize("kind", ["ez", "mz"])
def test_search_bf16x3_vs_f32_trunk(kind, monkeypatch):
    """Search-level effect of the default split-bf16 trunk: the same 256 x 50 search
    with the exact-f32 trunk and with bf16x3, same seeds. The trunks agree to f32 round-off per
    launch, so visit counts may differ only where a pUCT near-tie (within the 1e-6 epsilon of
    cselect_child) flips; the mismatch rate is reported and bounded, root values stay close.
    Conv-config search parity under the default is therefore tolerance-level, not bit-level
    (DESIGN.md §6.3); each precision's tree is bit-exact vs the oracle fed its own network outputs."""
    from lightzero_amd.mcts_ctree import EfficientZeroMCTSCtree, MuZeroMCTSCtree
    from lightzero_amd.utils import EasyDict
    B, S = 256, 50
    model = conv_model(kind, 11)
    cls = EfficientZeroMCTSCtree if kind == "ez" else MuZeroMCTSCtree
    res = {}
    for p in ("f32", "bf16x3"):
        monkeypatch.setenv("LZM_CONV_PRECISION", p)
        cfg = EasyDict(dict(num_simulations=S, discount_factor=0.997, device=DEV, lstm_horizon_len=5,
                            model=dict(support_scale=50 if kind == "ez" else 300, categorical_distribution=True)))
        res[p] = run_search(kind, B, S, seed=12, model=model, mcts=cls(cfg))
        oracle_replay(kind, res[p], B, S)
    differ = (res["f32"]["dist"] != res["bf16x3"]["dist"]).any(axis=1)
    rate = float(differ.mean())
    print(f"{kind}: roots whose visit counts differ between f32 and bf16x3 trunks: {int(differ.sum())}/{B} ({rate:.3f})")
    assert rate <= 0.1, rate
    # every root's first divergent walk: a near-tie moved by rounding, or a tie broken at a shifted
    # position of the glibc stream after an earlier root diverged (tests/divergence.py); reported to
    # $LZM_REPORT_DIR/divergence_conv_<kind>_bf16x3_vs_f32.json
    from tests.divergence import attribute, report
    rep = attribute(res["f32"], res["bf16x3"], B, S, res["f32"]["A"], ez=(kind == "ez"))
    report(f"conv_{kind}_bf16x3_vs_f32", rep)
    assert rep["first_divergence_kinds"].get("unexplained", 0) == 0, rep["first_divergences"][:5]
    assert rep["first_divergence_kinds"].get("tie_draw", 0) == 0
    same = ~differ
    np.testing.assert_allclose(res["bf16x3"]["values"][same], res["f32"]["values"][same], rtol=1e-3, atol=1e-3)


def test_ez_residency_refusal_falls_back_to_generic_with_same_results(monkeypatch):
    """lzm_search_conv_ez refuses a grid its static co-residency bound cannot hold (LZM_RESIDENCY_CUS caps
    the CU count it assumes) with LZM_ERR_RESIDENCY before running anything; EfficientZeroMCTSCtree.search
    then runs the generic path eagerly: the same visit counts, values and trajectories. Inside a stream
    capture the refusal is raised instead."""
    from lightzero_amd import _lib
    from lightzero_amd.mcts_ctree import EfficientZeroMCTSCtree
    from lightzero_amd.utils import EasyDict
    B, S = 48, 10
    model = conv_model("ez", 21)
    a = run_search("ez", B, S, seed=22, model=model, record=False)
    assert a["path"] == "fused"
    monkeypatch.setenv("LZM_RESIDENCY_CUS", "8")
    cfg = EasyDict(dict(num_simulations=S, discount_factor=0.997, device=DEV, lstm_horizon_len=5,
                        model=dict(support_scale=50, categorical_distribution=True)))
    mcts = EfficientZeroMCTSCtree(cfg)
    b = run_search("ez", B, S, seed=22, model=model, record=False, mcts=mcts)
    assert b["path"] == "generic (co-residency refused)" and mcts.residency_fallbacks == 1
    for key in ("dist", "values", "traj"):
        assert np.array_equal(a[key], b[key]), key
    # captured: raised, not a fallback inside the capture
    roots = EfficientZeroMCTSCtree.roots(B, [list(range(6))] * B)
    roots.prepare_no_noise([0.0] * B, a["logits0"].tolist(), [-1] * B)
    seeds = torch.arange(S, dtype=torch.int32, device=DEV)
    to_play = torch.full((B,), -1, dtype=torch.int32, device=DEV)
    roots.tree.reserve(S)  # (no allocation or host copy inside the capture)
    roots.tree.set_pb_c(19652, 1.25)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with pytest.raises(_lib.ResidencyError):
        with torch.cuda.graph(g):
            mcts.search(roots, model, a["lat0"], a["hidden0"], to_play, seeds=seeds)
    assert mcts.residency_fallbacks == 1


def test_ez_handoff_timeout_falls_back_to_generic_with_same_results():
    """another stream's kernel holds most CUs while the one-launch EZ search launches eagerly (the
    static occupancy bound accepted the grid): the resident workgroups' hand-off waits give up after 200 ms
    and abort the launch (error words 0 / 5), EfficientZeroMCTSCtree.search restores the tree it snapshotted
    and runs the generic path — the same visit counts, values and trajectories as an undisturbed search, the
    error words clear"""
    from lightzero_amd import _lib
    from lightzero_amd.mcts_ctree import EfficientZeroMCTSCtree
    from lightzero_amd.utils import EasyDict
    B, S = 64, 10
    model = conv_model("ez", 21)
    a = run_search("ez", B, S, seed=22, model=model, record=False)
    assert a["path"] == "fused"
    cfg = EasyDict(dict(num_simulations=S, discount_factor=0.997, device=DEV, lstm_horizon_len=5,
                        model=dict(support_scale=50, categorical_distribution=True)))
    mcts = EfficientZeroMCTSCtree(cfg)
    cus = torch.cuda.get_device_properties(DEV).multi_processor_count
    hog = torch.cuda.Stream(device=DEV)
    torch.cuda.synchronize()
    with torch.cuda.stream(hog):
        _lib.call("lzm_debug_hold_cus", cus - 40, 700000, _lib.stream_ptr(hog))  # 700 ms on all but 40 CUs
    b = run_search("ez", B, S, seed=22, model=model, record=False, mcts=mcts)
    torch.cuda.synchronize()
    print(f"path under a CU-holding kernel: {b['path']}, fallbacks {getattr(mcts, 'timeout_fallbacks', 0)}")
    assert b["path"] == "generic (hand-off timeout)" and mcts.timeout_fallbacks == 1
    for key in ("dist", "values", "traj"):
        assert np.array_equal(a[key], b[key]), key
