"""MuZeroModelMLP restated for PyTorch-ROCm (the network the CartPole search calls every simulation).

Reference: /root/reference/lzero/model/muzero_model_mlp.py:12-204 (model, ``initial_inference``,
``recurrent_inference``), ``DynamicsNetwork`` :327-440, and lzero/model/common.py
(``RepresentationNetworkMLP`` :467-517, ``PredictionNetworkMLP`` :883-971, ``SimNorm`` :53-91).
Every block there is built by DI-engine's ``MLP`` (not installed here); its construction is
restated in ``mlp()``: ``layer_num`` Linear layers with widths [in] + [hidden]*(layer_num-1) +
[out]; each hidden Linear is followed by BatchNorm1d then the activation; the last Linear is
followed by BatchNorm only if ``output_norm`` and the activation only if ``output_activation``;
``last_linear_layer_init_zero`` zeroes the last Linear's weight and bias.

Parity note: DI-engine is absent, so the network's numerics are not pinned to reference
outputs; the architecture, widths, init rules and forward order are.
"""
from dataclasses import dataclass
from typing import Optional, Sequence

import torch
import torch.nn as nn
import torch.nn.functional as F


@dataclass
class MZNetworkOutput:  # lzero/model/common.py:45-50
    value: torch.Tensor
    reward: torch.Tensor
    policy_logits: torch.Tensor
    latent_state: torch.Tensor


def mlp(in_channels: int, hidden_channels: int, out_channels: int, layer_num: int, activation: nn.Module,
        norm_type: Optional[str] = 'BN', output_activation: bool = True, output_norm: bool = True,
        last_linear_layer_init_zero: bool = False) -> nn.Sequential:
    channels = [in_channels] + [hidden_channels] * (layer_num - 1) + [out_channels]
    layers = []
    for i in range(layer_num - 1):
        layers.append(nn.Linear(channels[i], channels[i + 1]))
        if norm_type == 'BN':
            layers.append(nn.BatchNorm1d(channels[i + 1]))
        elif norm_type == 'LN':
            layers.append(nn.LayerNorm(channels[i + 1]))
        layers.append(activation)
    last = nn.Linear(channels[-2], channels[-1])
    layers.append(last)
    if output_norm and norm_type == 'BN':
        layers.append(nn.BatchNorm1d(channels[-1]))
    elif output_norm and norm_type == 'LN':
        layers.append(nn.LayerNorm(channels[-1]))
    if output_activation:
        layers.append(activation)
    if last_linear_layer_init_zero:
        nn.init.zeros_(last.weight)
        nn.init.zeros_(last.bias)
    return nn.Sequential(*layers)


class SimNorm(nn.Module):
    """Softmax over consecutive groups of ``dim`` features (common.py:53-91)."""

    def __init__(self, simnorm_dim: int) -> None:
        super().__init__()
        self.dim = simnorm_dim

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        shp = x.shape
        if shp[1] == 0:
            return x
        return F.softmax(x.view(*shp[:-1], -1, self.dim), dim=-1).view(*shp)


class RepresentationNetworkMLP(nn.Module):
    def __init__(self, observation_shape: int, hidden_channels: int = 64, layer_num: int = 2,
                 activation: nn.Module = nn.GELU(approximate='tanh'), norm_type: Optional[str] = 'BN',
                 group_size: int = 8):
        super().__init__()
        self.fc_representation = mlp(observation_shape, hidden_channels, hidden_channels, layer_num, activation,
                                     norm_type, output_activation=False, output_norm=False,
                                     last_linear_layer_init_zero=True)
        self.sim_norm = SimNorm(group_size)

    def forward(self, x):
        return self.sim_norm(self.fc_representation(x))


class PredictionNetworkMLP(nn.Module):
    def __init__(self, action_space_size: int, num_channels: int, common_layer_num: int = 2,
                 fc_value_layers: Sequence[int] = (32,), fc_policy_layers: Sequence[int] = (32,),
                 output_support_size: int = 601, last_linear_layer_init_zero: bool = True,
                 activation: nn.Module = nn.ReLU(inplace=True), norm_type: Optional[str] = 'BN'):
        super().__init__()
        self.fc_prediction_common = mlp(num_channels, num_channels, num_channels, common_layer_num, activation,
                                        norm_type, output_activation=True, output_norm=True)
        self.fc_value_head = mlp(num_channels, fc_value_layers[0], output_support_size, len(fc_value_layers) + 1,
                                 activation, norm_type, output_activation=False, output_norm=False,
                                 last_linear_layer_init_zero=last_linear_layer_init_zero)
        self.fc_policy_head = mlp(num_channels, fc_policy_layers[0], action_space_size, len(fc_policy_layers) + 1,
                                  activation, norm_type, output_activation=False, output_norm=False,
                                  last_linear_layer_init_zero=last_linear_layer_init_zero)

    def forward(self, latent_state):
        x = self.fc_prediction_common(latent_state)
        return self.fc_policy_head(x), self.fc_value_head(x)


class DynamicsNetwork(nn.Module):
    def __init__(self, action_encoding_dim: int = 2, num_channels: int = 64, common_layer_num: int = 2,
                 fc_reward_layers: Sequence[int] = (32,), output_support_size: int = 601,
                 last_linear_layer_init_zero: bool = True, activation: nn.Module = nn.ReLU(inplace=True),
                 norm_type: Optional[str] = 'BN', res_connection_in_dynamics: bool = False):
        super().__init__()
        self.action_encoding_dim = action_encoding_dim
        self.latent_state_dim = num_channels - action_encoding_dim
        self.res_connection_in_dynamics = res_connection_in_dynamics
        H = self.latent_state_dim
        if res_connection_in_dynamics:
            self.fc_dynamics_1 = mlp(num_channels, H, H, common_layer_num, activation, norm_type, True, True)
            self.fc_dynamics_2 = mlp(H, H, H, common_layer_num, activation, norm_type, True, True)
        else:
            self.fc_dynamics = mlp(num_channels, H, H, common_layer_num, activation, norm_type, True, True)
        self.fc_reward_head = mlp(H, fc_reward_layers[0], output_support_size, 2, activation, norm_type,
                                  output_activation=False, output_norm=False,
                                  last_linear_layer_init_zero=last_linear_layer_init_zero)

    def forward(self, state_action_encoding):
        if self.res_connection_in_dynamics:
            latent_state = state_action_encoding[:, :-self.action_encoding_dim]
            next_latent_state = self.fc_dynamics_1(state_action_encoding) + latent_state
            enc = self.fc_dynamics_2(next_latent_state)
        else:
            next_latent_state = self.fc_dynamics(state_action_encoding)
            enc = next_latent_state
        return next_latent_state, self.fc_reward_head(enc)


class MuZeroModelMLP(nn.Module):
    """MuZero for vector observations (muzero_model_mlp.py:12-204), discrete one-hot actions."""

    def __init__(self, observation_shape: int = 2, action_space_size: int = 6, latent_state_dim: int = 256,
                 fc_reward_layers=(32,), fc_value_layers=(32,), fc_policy_layers=(32,),
                 reward_support_size: int = 601, value_support_size: int = 601,
                 categorical_distribution: bool = True, last_linear_layer_init_zero: bool = True,
                 norm_type: Optional[str] = 'BN', res_connection_in_dynamics: bool = False, **kwargs):
        super().__init__()
        self.categorical_distribution = categorical_distribution
        self.reward_support_size = reward_support_size if categorical_distribution else 1
        self.value_support_size = value_support_size if categorical_distribution else 1
        self.action_space_size = action_space_size
        self.latent_state_dim = latent_state_dim
        self.representation_network = RepresentationNetworkMLP(observation_shape, latent_state_dim,
                                                               norm_type=norm_type)
        self.dynamics_network = DynamicsNetwork(action_space_size, latent_state_dim + action_space_size, 2,
                                                fc_reward_layers, self.reward_support_size,
                                                last_linear_layer_init_zero, norm_type=norm_type,
                                                res_connection_in_dynamics=res_connection_in_dynamics)
        self.prediction_network = PredictionNetworkMLP(action_space_size, latent_state_dim,
                                                       fc_value_layers=fc_value_layers,
                                                       fc_policy_layers=fc_policy_layers,
                                                       output_support_size=self.value_support_size,
                                                       last_linear_layer_init_zero=last_linear_layer_init_zero,
                                                       norm_type=norm_type)

    def initial_inference(self, obs: torch.Tensor) -> MZNetworkOutput:
        latent_state = self.representation_network(obs)
        policy_logits, value = self.prediction_network(latent_state)
        return MZNetworkOutput(value, [0. for _ in range(obs.size(0))], policy_logits, latent_state)

    def recurrent_inference(self, latent_state: torch.Tensor, action: torch.Tensor) -> MZNetworkOutput:
        a = action.long().reshape(-1, 1)
        one_hot = torch.zeros(a.shape[0], self.action_space_size, device=latent_state.device)
        one_hot.scatter_(1, a, 1)
        next_latent_state, reward = self.dynamics_network(torch.cat((latent_state, one_hot), dim=1))
        policy_logits, value = self.prediction_network(next_latent_state)
        return MZNetworkOutput(value, reward, policy_logits, next_latent_state)


def cartpole_muzero_model(random_heads: bool = True) -> MuZeroModelMLP:
    """The CartPole-v0 MuZero network (cartpole_muzero_config.py:31-39 over muzero.py defaults:
    latent 128, one-hot actions, BN, residual dynamics, support 601). ``random_heads`` keeps the
    last linear layers random instead of zero (a trained-net stand-in: zero heads make every
    simulation a tie)."""
    return MuZeroModelMLP(observation_shape=4, action_space_size=2, latent_state_dim=128,
                          categorical_distribution=True, last_linear_layer_init_zero=not random_heads,
                          norm_type='BN', res_connection_in_dynamics=True)
