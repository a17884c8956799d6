"""Convolutional MuZeroModel / EfficientZeroModel restated for PyTorch-ROCm (configs 3 and 5 of
BASELINE.json: Atari Pong EfficientZero and Atari Breakout MuZero, 64x64 stacked grey frames).

References (module and attribute names follow them, so a reference state_dict loads unchanged):
- ``MuZeroModel`` lzero/model/muzero_model.py:20-415 (``initial_inference`` :209, ``recurrent_inference``
  :241, ``_dynamics`` one-hot action planes :308-373) and its ``DynamicsNetwork`` :418-530;
- ``EfficientZeroModel`` lzero/model/efficientzero_model.py:20-423 and its LSTM value-prefix
  ``DynamicsNetwork`` :426-574;
- ``DownSample`` lzero/model/common.py:164-266, ``RepresentationNetwork`` :369-465,
  ``PredictionNetwork`` :744-881, ``EZNetworkOutput`` / ``MZNetworkOutput`` :35-50.
DI-engine's ``ResBlock`` (not installed) is restated from its known structure:
``basic``: conv3x3-BN-act, conv3x3-BN, + x, act; ``downsample``: conv3x3/2-BN-act, conv3x3-BN,
+ conv3x3/2(x) (no norm), act. All convolutions are bias-free except the 1x1 head convolutions.
DI-engine's ``MLP`` is ``model_mlp.mlp``.

Shapes at the Atari configs (observation (4, 64, 64), ``downsample=True``): conv3x3/2 4->32 (32x32),
basic(32), downsample 32->64 (16x16), basic(64), avgpool3/2 (8x8), basic(64), then
``num_res_blocks`` basic(64): latent 64x8x8 = 4096 floats. (SURVEY.md §8 lists the latent as
64x4x4; the reference computes ceil(64/8)^2 = 8x8 for 64x64 frames, efficientzero_model.py:120-123.)
Parity: DI-engine is absent, so outputs are not pinned to reference numbers; architecture, widths,
init rules and forward order are.
"""
import math
from dataclasses import dataclass
from typing import Optional, Sequence, Tuple

import torch
import torch.nn as nn

from .model_mlp import MZNetworkOutput, mlp


@dataclass
class EZNetworkOutput:  # lzero/model/common.py:35-42
    value: torch.Tensor
    value_prefix: torch.Tensor
    policy_logits: torch.Tensor
    latent_state: torch.Tensor
    reward_hidden_state: Tuple[torch.Tensor, torch.Tensor]


def _norm2d(norm_type, channels, hw):
    if norm_type == 'BN':
        return nn.BatchNorm2d(channels)
    return nn.LayerNorm([channels, *hw], eps=1e-5)


class ResBlock(nn.Module):
    """DI-engine ResBlock(res_type in {'basic', 'downsample'}, bias=False), BatchNorm only."""

    def __init__(self, in_channels: int, activation: nn.Module, out_channels: Optional[int] = None,
                 res_type: str = 'basic'):
        super().__init__()
        out_channels = in_channels if out_channels is None else out_channels
        stride = 2 if res_type == 'downsample' else 1
        self.res_type = res_type
        self.conv1 = nn.Conv2d(in_channels, out_channels, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(out_channels)
        self.conv2 = nn.Conv2d(out_channels, out_channels, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(out_channels)
        if res_type == 'downsample':
            self.conv3 = nn.Conv2d(in_channels, out_channels, 3, 2, 1, bias=False)
        self.act = activation

    def forward(self, x):
        identity = self.conv3(x) if self.res_type == 'downsample' else x
        y = self.act(self.bn1(self.conv1(x)))
        y = self.bn2(self.conv2(y))
        return self.act(y + identity)


class DownSample(nn.Module):
    """common.py:164-266 (BN variant)."""

    def __init__(self, observation_shape: Sequence[int], out_channels: int, activation: nn.Module):
        super().__init__()
        self.observation_shape = observation_shape
        half = out_channels // 2
        self.conv1 = nn.Conv2d(observation_shape[0], half, 3, 2, 1, bias=False)
        self.norm1 = nn.BatchNorm2d(half)
        self.resblocks1 = nn.ModuleList([ResBlock(half, activation)])
        self.downsample_block = ResBlock(half, activation, out_channels, 'downsample')
        self.resblocks2 = nn.ModuleList([ResBlock(out_channels, activation)])
        self.pooling1 = nn.AvgPool2d(kernel_size=3, stride=2, padding=1)
        self.resblocks3 = nn.ModuleList([ResBlock(out_channels, activation)])
        self.pooling2 = nn.AvgPool2d(kernel_size=3, stride=2, padding=1)
        self.activation = activation

    def forward(self, x):
        x = self.activation(self.norm1(self.conv1(x)))
        for b in self.resblocks1:
            x = b(x)
        x = self.downsample_block(x)
        for b in self.resblocks2:
            x = b(x)
        x = self.pooling1(x)
        for b in self.resblocks3:
            x = b(x)
        if self.observation_shape[1] == 96:
            x = self.pooling2(x)
        return x


class RepresentationNetwork(nn.Module):
    """common.py:369-465 (use_sim_norm=False, as MuZeroModel / EfficientZeroModel build it)."""

    def __init__(self, observation_shape, num_res_blocks, num_channels, downsample, activation, norm_type='BN'):
        super().__init__()
        self.downsample = downsample
        if downsample:
            self.downsample_net = DownSample(observation_shape, num_channels, activation)
        else:
            self.conv = nn.Conv2d(observation_shape[0], num_channels, 3, 1, 1, bias=False)
            self.norm = _norm2d(norm_type, num_channels, observation_shape[-2:])
        self.resblocks = nn.ModuleList([ResBlock(num_channels, activation) for _ in range(num_res_blocks)])
        self.activation = activation

    def forward(self, x):
        if self.downsample:
            x = self.downsample_net(x)
        else:
            x = self.activation(self.norm(self.conv(x)))
        for b in self.resblocks:
            x = b(x)
        return x


class PredictionNetwork(nn.Module):
    """common.py:744-881."""

    def __init__(self, action_space_size, num_res_blocks, num_channels, value_head_channels, policy_head_channels,
                 fc_value_layers, fc_policy_layers, output_support_size, flatten_value, flatten_policy, activation,
                 last_linear_layer_init_zero=True, norm_type='BN'):
        super().__init__()
        self.resblocks = nn.ModuleList([ResBlock(num_channels, activation) for _ in range(num_res_blocks)])
        self.conv1x1_value = nn.Conv2d(num_channels, value_head_channels, 1)
        self.conv1x1_policy = nn.Conv2d(num_channels, policy_head_channels, 1)
        self.norm_value = nn.BatchNorm2d(value_head_channels)
        self.norm_policy = nn.BatchNorm2d(policy_head_channels)
        self.flatten_output_size_for_value_head = flatten_value
        self.flatten_output_size_for_policy_head = flatten_policy
        self.activation = activation
        self.fc_value = mlp(flatten_value, fc_value_layers[0], output_support_size, len(fc_value_layers) + 1,
                            activation, norm_type, output_activation=False, output_norm=False,
                            last_linear_layer_init_zero=last_linear_layer_init_zero)
        self.fc_policy = mlp(flatten_policy, fc_policy_layers[0], action_space_size, len(fc_policy_layers) + 1,
                             activation, norm_type, output_activation=False, output_norm=False,
                             last_linear_layer_init_zero=last_linear_layer_init_zero)

    def forward(self, latent_state):
        for b in self.resblocks:
            latent_state = b(latent_state)
        value = self.activation(self.norm_value(self.conv1x1_value(latent_state)))
        policy = self.activation(self.norm_policy(self.conv1x1_policy(latent_state)))
        value = self.fc_value(value.reshape(-1, self.flatten_output_size_for_value_head))
        policy = self.fc_policy(policy.reshape(-1, self.flatten_output_size_for_policy_head))
        return policy, value


class _DynamicsTrunk(nn.Module):
    """The part shared by muzero_model.py:418-530 and efficientzero_model.py:426-574: conv3x3 over
    [latent | action planes] -> BN, + latent (residual), act, res blocks, then the 1x1 reward conv."""

    def __init__(self, action_encoding_dim, num_res_blocks, num_channels, reward_head_channels, activation):
        super().__init__()
        assert num_channels > action_encoding_dim
        self.action_encoding_dim = action_encoding_dim
        self.num_channels = num_channels
        c = num_channels - action_encoding_dim
        self.conv = nn.Conv2d(num_channels, c, 3, 1, 1, bias=False)
        self.norm_common = nn.BatchNorm2d(c)
        self.resblocks = nn.ModuleList([ResBlock(c, activation) for _ in range(num_res_blocks)])
        self.conv1x1_reward = nn.Conv2d(c, reward_head_channels, 1)
        self.norm_reward = nn.BatchNorm2d(reward_head_channels)
        self.activation = activation

    def trunk(self, state_action_encoding):
        state_encoding = state_action_encoding[:, :-self.action_encoding_dim, :, :]
        x = self.norm_common(self.conv(state_action_encoding))
        x = self.activation(x + state_encoding)
        for b in self.resblocks:
            x = b(x)
        r = self.activation(self.norm_reward(self.conv1x1_reward(x)))
        return x, r


class DynamicsNetwork(_DynamicsTrunk):
    """MuZero dynamics (muzero_model.py:418-530): reward head MLP over the flattened reward planes."""

    def __init__(self, action_encoding_dim, num_res_blocks, num_channels, reward_head_channels, fc_reward_layers,
                 output_support_size, flatten_reward, activation, last_linear_layer_init_zero=True, norm_type='BN'):
        super().__init__(action_encoding_dim, num_res_blocks, num_channels, reward_head_channels, activation)
        self.flatten_output_size_for_reward_head = flatten_reward
        self.fc_reward_head = mlp(flatten_reward, fc_reward_layers[0], output_support_size, len(fc_reward_layers) + 1,
                                  activation, norm_type, output_activation=False, output_norm=False,
                                  last_linear_layer_init_zero=last_linear_layer_init_zero)

    def forward(self, state_action_encoding):
        x, r = self.trunk(state_action_encoding)
        return x, self.fc_reward_head(r.view(r.shape[0], -1))


class EZDynamicsNetwork(_DynamicsTrunk):
    """EfficientZero dynamics (efficientzero_model.py:426-574): LSTM over the flattened reward
    planes, BatchNorm1d + act on its output, then the value-prefix MLP."""

    def __init__(self, action_encoding_dim, num_res_blocks, num_channels, reward_head_channels, fc_reward_layers,
                 output_support_size, flatten_reward, lstm_hidden_size, activation, last_linear_layer_init_zero=True,
                 norm_type='BN'):
        super().__init__(action_encoding_dim, num_res_blocks, num_channels, reward_head_channels, activation)
        self.flatten_output_size_for_reward_head = flatten_reward
        self.lstm_hidden_size = lstm_hidden_size
        self.lstm = nn.LSTM(input_size=flatten_reward, hidden_size=lstm_hidden_size)
        self.norm_value_prefix = nn.BatchNorm1d(lstm_hidden_size)
        self.fc_reward_head = mlp(lstm_hidden_size, fc_reward_layers[0], output_support_size,
                                  len(fc_reward_layers) + 1, activation, norm_type, output_activation=False,
                                  output_norm=False, last_linear_layer_init_zero=last_linear_layer_init_zero)

    def forward(self, state_action_encoding, reward_hidden_state):
        x, r = self.trunk(state_action_encoding)
        r = r.reshape(-1, self.flatten_output_size_for_reward_head).unsqueeze(0)
        value_prefix, next_hidden = self.lstm(r, reward_hidden_state)
        value_prefix = self.activation(self.norm_value_prefix(value_prefix.squeeze(0)))
        return x, next_hidden, self.fc_reward_head(value_prefix)


def _latent_size(observation_shape, downsample):
    if not downsample:
        return observation_shape[1] * observation_shape[2]
    if observation_shape[1] == 96:
        return math.ceil(observation_shape[1] / 16) * math.ceil(observation_shape[2] / 16)
    return math.ceil(observation_shape[1] / 8) * math.ceil(observation_shape[2] / 8)


def _action_planes(action, A, latent_state):
    """one-hot action expanded over the latent plane (muzero_model.py:330-345)"""
    a = action.reshape(-1, 1).long()
    one_hot = torch.zeros(a.shape[0], A, device=action.device)
    one_hot.scatter_(1, a, 1)
    return one_hot.unsqueeze(-1).unsqueeze(-1).expand(latent_state.shape[0], A, latent_state.shape[2],
                                                      latent_state.shape[3])


class _ConvModelBase(nn.Module):
    def _build(self, observation_shape, action_space_size, num_res_blocks, num_channels, reward_head_channels,
               value_head_channels, policy_head_channels, fc_value_layers, fc_policy_layers, value_support_size,
               downsample, activation, last_linear_layer_init_zero, norm_type, self_supervised_learning_loss,
               proj_hid, proj_out, pred_hid, pred_out):
        self.action_space_size = action_space_size
        self.action_encoding_dim = action_space_size
        self.downsample = downsample
        latent = _latent_size(observation_shape, downsample)
        self.latent_hw = (int(math.sqrt(latent)),) * 2
        self.representation_network = RepresentationNetwork(observation_shape, num_res_blocks, num_channels,
                                                            downsample, activation, norm_type)
        self.prediction_network = PredictionNetwork(action_space_size, num_res_blocks, num_channels,
                                                    value_head_channels, policy_head_channels, fc_value_layers,
                                                    fc_policy_layers, value_support_size,
                                                    value_head_channels * latent, policy_head_channels * latent,
                                                    activation, last_linear_layer_init_zero, norm_type)
        self.self_supervised_learning_loss = self_supervised_learning_loss
        if self_supervised_learning_loss:
            d = num_channels * latent
            self.projection = nn.Sequential(
                nn.Linear(d, proj_hid), nn.BatchNorm1d(proj_hid), activation,
                nn.Linear(proj_hid, proj_hid), nn.BatchNorm1d(proj_hid), activation,
                nn.Linear(proj_hid, proj_out), nn.BatchNorm1d(proj_out))
            self.prediction_head = nn.Sequential(
                nn.Linear(proj_out, pred_hid), nn.BatchNorm1d(pred_hid), activation, nn.Linear(pred_hid, pred_out))
        return reward_head_channels * latent

    def _prediction(self, latent_state):
        return self.prediction_network(latent_state)

    def _encode(self, latent_state, action):
        return torch.cat((latent_state, _action_planes(action, self.action_space_size, latent_state)), dim=1)

    def project(self, latent_state, with_grad=True):
        proj = self.projection(latent_state.reshape(latent_state.shape[0], -1))
        return self.prediction_head(proj) if with_grad else proj.detach()


class MuZeroModel(_ConvModelBase):
    """lzero/model/muzero_model.py:20-415 (one-hot action encoding, state_norm=False)."""

    def __init__(self, observation_shape=(12, 96, 96), action_space_size=6, num_res_blocks=1, num_channels=64,
                 reward_head_channels=16, value_head_channels=16, policy_head_channels=16,
                 fc_reward_layers=(32,), fc_value_layers=(32,), fc_policy_layers=(32,), reward_support_size=601,
                 value_support_size=601, proj_hid=1024, proj_out=1024, pred_hid=512, pred_out=1024,
                 self_supervised_learning_loss=False, categorical_distribution=True,
                 activation: nn.Module = nn.ReLU(inplace=True), last_linear_layer_init_zero=True, downsample=False,
                 norm_type='BN', **kwargs):
        super().__init__()
        if not categorical_distribution:
            reward_support_size = value_support_size = 1
        flat_r = self._build(observation_shape, action_space_size, num_res_blocks, num_channels, reward_head_channels,
                             value_head_channels, policy_head_channels, fc_value_layers, fc_policy_layers,
                             value_support_size, downsample, activation, last_linear_layer_init_zero, norm_type,
                             self_supervised_learning_loss, proj_hid, proj_out, pred_hid, pred_out)
        self.dynamics_network = DynamicsNetwork(action_space_size, num_res_blocks, num_channels + action_space_size,
                                                reward_head_channels, fc_reward_layers, reward_support_size, flat_r,
                                                activation, last_linear_layer_init_zero, norm_type)

    def initial_inference(self, obs):
        latent_state = self.representation_network(obs)
        policy_logits, value = self._prediction(latent_state)
        return MZNetworkOutput(value, [0. for _ in range(obs.size(0))], policy_logits, latent_state)

    def recurrent_inference(self, latent_state, action):
        next_latent_state, reward = self.dynamics_network(self._encode(latent_state, action))
        policy_logits, value = self._prediction(next_latent_state)
        return MZNetworkOutput(value, reward, policy_logits, next_latent_state)


class EfficientZeroModel(_ConvModelBase):
    """lzero/model/efficientzero_model.py:20-423 (one-hot action encoding, state_norm=False)."""

    def __init__(self, observation_shape=(12, 96, 96), action_space_size=6, lstm_hidden_size=512, num_res_blocks=1,
                 num_channels=64, reward_head_channels=16, value_head_channels=16, policy_head_channels=16,
                 fc_reward_layers=(32,), fc_value_layers=(32,), fc_policy_layers=(32,), reward_support_size=601,
                 value_support_size=601, proj_hid=1024, proj_out=1024, pred_hid=512, pred_out=1024,
                 self_supervised_learning_loss=True, categorical_distribution=True, last_linear_layer_init_zero=True,
                 downsample=False, activation: nn.Module = nn.ReLU(inplace=True), norm_type='BN', **kwargs):
        super().__init__()
        if not categorical_distribution:
            reward_support_size = value_support_size = 1
        self.lstm_hidden_size = lstm_hidden_size
        flat_r = self._build(observation_shape, action_space_size, num_res_blocks, num_channels, reward_head_channels,
                             value_head_channels, policy_head_channels, fc_value_layers, fc_policy_layers,
                             value_support_size, downsample, activation, last_linear_layer_init_zero, norm_type,
                             self_supervised_learning_loss, proj_hid, proj_out, pred_hid, pred_out)
        self.dynamics_network = EZDynamicsNetwork(action_space_size, num_res_blocks, num_channels + action_space_size,
                                                  reward_head_channels, fc_reward_layers, reward_support_size, flat_r,
                                                  lstm_hidden_size, activation, last_linear_layer_init_zero, norm_type)

    def initial_inference(self, obs):
        B = obs.size(0)
        latent_state = self.representation_network(obs)
        policy_logits, value = self._prediction(latent_state)
        z = torch.zeros(1, B, self.lstm_hidden_size, device=obs.device)
        return EZNetworkOutput(value, [0. for _ in range(B)], policy_logits, latent_state, (z, z.clone()))

    def recurrent_inference(self, latent_state, reward_hidden_state, action):
        nxt, hidden, value_prefix = self.dynamics_network(self._encode(latent_state, action), reward_hidden_state)
        policy_logits, value = self._prediction(nxt)
        return EZNetworkOutput(value, value_prefix, policy_logits, nxt, hidden)


def atari_efficientzero_model(action_space_size=6, **kw):
    """zoo/atari/config/atari_efficientzero_config.py:38-52 (Pong: 6 actions, support 101)."""
    args = dict(observation_shape=(4, 64, 64), action_space_size=action_space_size, downsample=True,
                self_supervised_learning_loss=True, norm_type='BN', reward_support_size=101, value_support_size=101)
    args.update(kw)
    return EfficientZeroModel(**args)


def atari_muzero_model(action_space_size=4, **kw):
    """zoo/atari/config/atari_muzero_config.py:49-63 (Breakout: 4 actions, support 601)."""
    args = dict(observation_shape=(4, 64, 64), action_space_size=action_space_size, downsample=True,
                self_supervised_learning_loss=True, norm_type='BN')
    args.update(kw)
    return MuZeroModel(**args)
