"""initial_inference in one launch (lightzero_amd.initial, csrc/lzm_initial.h).

CPU: the BN-folded layer list evaluated with torch equals the module's initial_inference (pins the
folding and the layer order the kernel reads). GPU: lzm_mlp_initial_inference equals the module
within fp32 tolerance (rtol 1e-4, atol 1e-5) at a ragged and the bench batch, random and
reference zero-init heads, and re-folds in place after a parameter update.
The network itself is restated (DI-engine absent): parity unpinned against reference outputs.
"""
import pytest
import torch
import torch.nn.functional as F

from lightzero_amd.initial import describe_initial
from lightzero_amd.model_mlp import cartpole_muzero_model


def _model(seed, random_heads=True, device="cpu"):
    torch.manual_seed(seed)
    m = cartpole_muzero_model(random_heads=random_heads)
    g = torch.Generator().manual_seed(seed + 1)
    for mod in m.modules():  # non-trivial eval-mode BatchNorm statistics
        if isinstance(mod, torch.nn.BatchNorm1d):
            n = mod.num_features
            mod.running_mean.copy_(torch.randn(n, generator=g) * 0.1)
            mod.running_var.copy_(torch.rand(n, generator=g) + 0.5)
            mod.weight.data.copy_(torch.rand(n, generator=g) + 0.5)
            mod.bias.data.copy_(torch.randn(n, generator=g) * 0.1)
    if random_heads:  # the representation's last Linear is zero-init in the reference: give it values
        last = m.representation_network.fc_representation[-1]
        last.weight.data.copy_(torch.randn(last.weight.shape, generator=g) * 0.1)
        last.bias.data.copy_(torch.randn(last.bias.shape, generator=g) * 0.1)
    return m.to(device).eval()


def _folded_forward(layers, dims, obs):
    def lin(x, l):
        W, b = layers[l]
        return F.linear(x, W, b)
    x = F.gelu(lin(obs, 0), approximate="tanh")
    x = lin(x, 1)
    B, H, G = x.shape[0], dims["hidden"], dims["group"]
    lat = torch.softmax(x.view(B, H // G, G), dim=-1).view(B, H)
    p = torch.relu(lin(torch.relu(lin(lat, 2)), 3))
    value = lin(torch.relu(lin(p, 4)), 5)
    policy = lin(torch.relu(lin(p, 6)), 7)
    return lat, value, policy


def test_folded_initial_layers_match_module():
    m = _model(3)
    layers, dims = describe_initial(m)
    assert dims == dict(obs=4, hidden=128, head_hidden=32, support=601, actions=2, group=8)
    obs = torch.randn(33, 4, generator=torch.Generator().manual_seed(0))
    with torch.no_grad():
        ref = m.initial_inference(obs)
        lat, value, policy = _folded_forward(layers, dims, obs)
    torch.testing.assert_close(lat, ref.latent_state, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(value, ref.value, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(policy, ref.policy_logits, rtol=1e-4, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("B,random_heads", [(37, True), (256, True), (64, False)])
def test_fused_initial_inference_matches_module(B, random_heads):
    from lightzero_amd.initial import FusedInitialInference
    dev = torch.device("cuda", 0)
    m = _model(5, random_heads, dev)
    fi = FusedInitialInference(m)
    obs = torch.randn(B, 4, generator=torch.Generator(device=dev).manual_seed(1), device=dev)
    with torch.no_grad():
        ref = m.initial_inference(obs)
        got = fi.initial_inference(obs)
    torch.testing.assert_close(got.latent_state, ref.latent_state, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(got.value, ref.value, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(got.policy_logits, ref.policy_logits, rtol=1e-4, atol=1e-5)
    # a parameter update is picked up (re-folded in place)
    flat = fi.flat
    with torch.no_grad():
        m.prediction_network.fc_policy_head[-1].bias.add_(1.0)
        ref2 = m.initial_inference(obs)
        got2 = fi.initial_inference(obs)
    assert fi.flat is flat
    torch.testing.assert_close(got2.policy_logits, ref2.policy_logits, rtol=1e-4, atol=1e-5)
