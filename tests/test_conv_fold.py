"""CPU: the BN-folded recurrent step (lightzero_amd.conv_infer) equals the conv module's own forward.

Float32 on both sides; folding reorders the BatchNorm arithmetic, so the comparison is within
float32 rounding (rtol 1e-4, atol 1e-5 on logits and latents). Also: in-place re-folding after a
parameter update, and rejection of models the fold does not recognise.
"""
import pytest
import torch

from lightzero_amd.conv_infer import FoldedCache, FoldedConvNet, NotFoldable, fold_tensors
from lightzero_amd.model_conv import atari_efficientzero_model, atari_muzero_model


def _model(kind, seed=0):
    torch.manual_seed(seed)
    m = (atari_efficientzero_model if kind == "ez" else atari_muzero_model)(last_linear_layer_init_zero=False)
    g = torch.Generator().manual_seed(seed + 1)
    for mod in m.modules():
        if isinstance(mod, (torch.nn.BatchNorm1d, torch.nn.BatchNorm2d)):
            n = mod.num_features
            mod.running_mean.copy_(torch.randn(n, generator=g) * 0.1)
            mod.running_var.copy_(torch.rand(n, generator=g) + 0.5)
            mod.weight.data.copy_(torch.rand(n, generator=g) + 0.5)
            mod.bias.data.copy_(torch.randn(n, generator=g) * 0.1)
    return m.eval()


def _compare(kind, m, net, B=6, seed=0):
    g = torch.Generator().manual_seed(seed)
    lat = torch.relu(torch.randn(B, 64, 8, 8, generator=g))
    act = torch.randint(0, m.action_space_size, (B,), generator=g)
    with torch.no_grad():
        if kind == "ez":
            hc = (torch.randn(1, B, 512, generator=g) * 0.5, torch.randn(1, B, 512, generator=g) * 0.5)
            ref, got = m.recurrent_inference(lat, hc, act), net.recurrent_inference(lat, hc, act)
            torch.testing.assert_close(got.value_prefix, ref.value_prefix, rtol=1e-4, atol=1e-5)
            for a, b in zip(got.reward_hidden_state, ref.reward_hidden_state):
                torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5)
        else:
            ref, got = m.recurrent_inference(lat, act), net.recurrent_inference(lat, act)
            torch.testing.assert_close(got.reward, ref.reward, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(got.latent_state, ref.latent_state, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(got.value, ref.value, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(got.policy_logits, ref.policy_logits, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("kind", ["ez", "mz"])
def test_folded_recurrent_step_matches_module(kind):
    m = _model(kind)
    _compare(kind, m, FoldedConvNet(m))


@pytest.mark.parametrize("kind", ["ez", "mz"])
def test_refold_in_place_after_update(kind):
    m = _model(kind)
    cache = FoldedCache()
    net = cache.get(m)
    ptrs = {k: v.data_ptr() for k, v in net.t.items()}
    with torch.no_grad():
        for p in m.parameters():
            p.mul_(0.9)
        m.dynamics_network.norm_common.running_var.mul_(1.5)
    assert cache.get(m) is net
    assert {k: v.data_ptr() for k, v in net.t.items()} == ptrs
    _compare(kind, m, net, seed=1)


def test_fold_rejects_unrecognised_models():
    from lightzero_amd.model_mlp import MuZeroModelMLP
    assert FoldedCache().get(MuZeroModelMLP(observation_shape=4, action_space_size=2)) is None
    m = _model("mz")
    m.dynamics_network.resblocks[0].res_type = "bottleneck"
    with pytest.raises(NotFoldable):
        fold_tensors(m)
