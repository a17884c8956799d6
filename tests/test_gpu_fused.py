"""GPU: the fused whole-search kernel (lzm_search_mlp) with MuZeroModelMLP networks.

1. Tree parity: every simulation's requests (x, last action, search_len) and the final visit
   distributions, root values and trajectories equal the oracle's when the oracle is fed the
   decoded values and policy logits the fused network produced (recorded per simulation) —
   bit-exact, in parity (glibc) and fast (Philox) modes, with zero-init heads (all-tie search,
   exercises the serial resolution of ties that reach expanded children), 2-player, a partial
   last slice, and a tree too large for LDS (HBM-resident slice).
2. Network parity: the fused recurrent_inference + decode vs the PyTorch module on the same
   gathered latents (BatchNorm folded, fp32 FMA): latents/logits rtol 1e-4 / atol 1e-5;
   decoded reward/value atol 1e-5 * support_scale (summation-order bound over the support).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from oracle.oracle import OracleTree  # noqa: E402
from tests.helpers import DISC, NOISE_W, PB_C_BASE, PB_C_INIT, VDM  # noqa: E402
from tests.test_gpu_numerics import torch_inverse_scalar_transform  # noqa: E402

DEV = torch.device("cuda", 0)


def make_model(A, H, zero_heads, seed=0, support_scale=300):
    from lightzero_amd.model_mlp import MuZeroModelMLP
    torch.manual_seed(seed)
    m = MuZeroModelMLP(observation_shape=4, action_space_size=A, latent_state_dim=H, categorical_distribution=True,
                       reward_support_size=2 * support_scale + 1, value_support_size=2 * support_scale + 1,
                       last_linear_layer_init_zero=zero_heads, norm_type='BN', res_connection_in_dynamics=True)
    g = torch.Generator().manual_seed(seed + 1)
    for mod in m.modules():
        if isinstance(mod, torch.nn.BatchNorm1d):
            with torch.no_grad():
                mod.running_mean.copy_(torch.randn(mod.running_mean.shape, generator=g) * 0.1)
                mod.running_var.copy_(torch.rand(mod.running_var.shape, generator=g) * 0.5 + 0.75)
    return m.to(DEV).eval()


def fused_search(B, S, A, H, zero_heads, players, fast, seed, support_scale=300):
    from lightzero_amd.mcts_ctree import MuZeroMCTSCtree
    from lightzero_amd.tree import SequentialSeeds, set_seed_source
    from lightzero_amd.utils import EasyDict
    model = make_model(A, H, zero_heads, seed, support_scale)
    rng = np.random.default_rng(seed)
    obs = torch.from_numpy(rng.normal(size=(B, 4)).astype(np.float32)).to(DEV)
    with torch.no_grad():
        out = model.initial_inference(obs)
    logits0 = out.policy_logits.float().cpu().numpy()
    noises = rng.dirichlet([0.3] * A, size=B).astype(np.float32)
    to_play = [-1] * B if players == 1 else rng.integers(1, 3, size=B).tolist()
    cfg = EasyDict(dict(num_simulations=S, discount_factor=float(DISC), device=DEV,
                        model=dict(support_scale=support_scale, categorical_distribution=True)))
    cls = MuZeroMCTSCtree
    old = cls.rng_mode
    cls.rng_mode = "philox" if fast else "glibc"
    try:
        mcts = cls(cfg)
        mcts.record = True
        roots = cls.roots(B, [list(range(A))] * B)
        roots.prepare(float(NOISE_W), [n.tolist() for n in noises], [0.0] * B, logits0.tolist(), to_play)
        set_seed_source(SequentialSeeds(seed))
        try:
            mcts.search(roots, model, out.latent_state, to_play)
        finally:
            set_seed_source(None)
        assert mcts._fused(model, roots.tree) is not None, "model should take the fused path"
        rec = mcts.last_record.numpy()
        t = roots.tree
        res = dict(rec=rec, dist=t.distributions().cpu().numpy(), values=t.values().cpu().numpy(),
                   traj=t.trajectories(S + 2).cpu().numpy(), pool=mcts._buf.pool.clone(), diag=t.search_diagnostics(),
                   model=model, logits0=logits0, noises=noises, to_play=np.array(to_play, np.int32))
        roots.clear()
        return res
    finally:
        cls.rng_mode = old


CASES = [
    # B, S, A, H, zero_heads, players, fast
    (256, 50, 2, 128, False, 1, False),
    (256, 50, 2, 128, True, 1, False),
    (100, 40, 3, 64, False, 2, False),
    (64, 50, 9, 64, False, 1, False),   # cap = 460 nodes: slice stays in HBM
    (256, 50, 2, 128, False, 1, True),
    (96, 30, 4, 64, True, 2, True),
    (1, 10, 2, 128, False, 1, False),    # edge sizes: one root; a long search; a batch past one root per CU
    (8, 100, 2, 128, False, 1, False),
    (1024, 20, 2, 128, False, 1, False),
]


def _case_id(c):
    return "b{}_s{}_a{}_h{}_{}_p{}_{}".format(c[0], c[1], c[2], c[3], "zero" if c[4] else "rand", c[5],
                                              "philox" if c[6] else "glibc")


@pytest.mark.parametrize("case", CASES, ids=_case_id)
def test_fused_tree_exact_given_network_outputs(case):
    check_tree_exact(case)


# every roots-per-workgroup variant of the kernel (the library picks one from the batch size)
@pytest.mark.parametrize("roots", [1, 2, 4, 8])
@pytest.mark.parametrize("case", [CASES[0], CASES[2], CASES[3], CASES[5]], ids=_case_id)
def test_fused_roots_per_workgroup(case, roots, monkeypatch):
    monkeypatch.setenv("LZM_ROOTS_PER_WG", str(roots))
    check_tree_exact(case)


# the config-2 shape takes the network-resident kernel (lzm_search_res.h); the same cases through
# the weight-streaming kernel (LZM_FUSED_RES=0) and the speculative two-row variant (LZM_RES_SPEC=1)
@pytest.mark.parametrize("env", ["LZM_FUSED_RES=0", "LZM_RES_SPEC=1", "LZM_RES_SELECT=0", "LZM_RES_SELECT=2",
                                 "LZM_RES_SELECT=3", "LZM_RES_SPEC_DEPTH=0"])
@pytest.mark.parametrize("case", [CASES[0], CASES[1], CASES[4]], ids=_case_id)
def test_fused_kernel_variants(case, env, monkeypatch):
    k, v = env.split("=")
    monkeypatch.setenv(k, v)
    check_tree_exact(case)


def test_zero_heads_depth_speculation_exercised():
    """Zero-init heads tie between visited children often: the resident kernel publishes such a
    root's depth early when every draw outcome gives the same depth (speculate_depth_a2), and the
    tree stays bit-exact with the oracle (check_tree_exact)."""
    r = check_tree_exact(CASES[1])
    assert r["diag"][2] > 0, "no tie was resolved through depth speculation"


def test_resident_kernel_serves_config2():
    from lightzero_amd import _lib
    L = _lib.load()
    assert L.lzm_search_mlp_kind(256, 2, 128, 32, 601, 1) == 1
    assert L.lzm_search_mlp_kind(256, 2, 64, 32, 601, 1) == 0   # other shapes: weight-streaming kernel
    assert L.lzm_search_mlp_kind(4096, 2, 128, 32, 601, 1) == 0  # several roots per workgroup


def check_tree_exact(case):
    B, S, A, H, zero, players, fast = case
    r = fused_search(B, S, A, H, zero, players, fast, seed=B + S + A)
    rec = r["rec"]
    assert r["diag"][0] == 0, "look-back spin timeout or depth speculation mismatch"
    assert r["diag"][3] == 0, "depth speculation mismatch"
    ot = OracleTree(B, A, S, fast_rng=fast)
    ot.set_delta(VDM)
    ot.prepare(NOISE_W, r["noises"], np.zeros(B, np.float32), r["logits0"], r["to_play"])
    for k in range(S):
        x, y, a, vtp, slen = ot.traverse(PB_C_BASE, PB_C_INIT, DISC, int(rec["seeds"][k]), r["to_play"])
        assert np.array_equal(x, rec["x"][k]), f"x differs at sim {k}"
        assert np.array_equal(a, rec["action"][k]), f"action differs at sim {k}"
        assert np.array_equal(slen, rec["search_len"][k]), f"search_len differs at sim {k}"
        ot.backprop(k + 1, DISC, rec["decoded"][k][:, 0], rec["decoded"][k][:, 1], rec["policy_logits"][k], vtp)
    assert np.array_equal(r["dist"], ot.distributions())
    assert np.array_equal(r["values"], ot.values())
    assert np.array_equal(r["traj"], ot.trajectories(S + 2))
    return r


# support 601 decodes from registers across the workgroup; support 21 (< 512 lanes) through LDS
@pytest.mark.parametrize("H,A,scale", [(128, 2, 300), (64, 9, 300), (64, 3, 10)])
def test_fused_network_matches_torch_module(H, A, scale):
    B, S = 128, 20
    r = fused_search(B, S, A, H, False, 1, False, seed=3, support_scale=scale)
    rec, pool, model = r["rec"], r["pool"], r["model"]
    idx = torch.arange(B, device=DEV)
    with torch.no_grad():
        for k in range(S):
            x = torch.from_numpy(rec["x"][k]).long().to(DEV)
            lat = pool[x, idx]
            out = model.recurrent_inference(lat, torch.from_numpy(rec["action"][k]).long().to(DEV))
            torch.testing.assert_close(pool[k + 1], out.latent_state, rtol=1e-4, atol=1e-5)
            torch.testing.assert_close(torch.from_numpy(rec["policy_logits"][k]).to(DEV), out.policy_logits,
                                       rtol=1e-4, atol=1e-5)
            dec = torch.from_numpy(rec["decoded"][k]).to(DEV)
            torch.testing.assert_close(dec[:, 0], torch_inverse_scalar_transform(out.reward, scale).squeeze(1),
                                       rtol=1e-4, atol=1e-5 * scale)
            torch.testing.assert_close(dec[:, 1], torch_inverse_scalar_transform(out.value, scale).squeeze(1),
                                       rtol=1e-4, atol=1e-5 * scale)


def test_fused_pack_rejects_unsupported_models():
    from lightzero_amd.fused import NotPackable, describe
    from tests.test_gpu_search import CategoricalModel
    with pytest.raises(NotPackable):
        describe(CategoricalModel())
