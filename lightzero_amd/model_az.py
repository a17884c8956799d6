"""AlphaZeroModel restated for PyTorch-ROCm (the policy-value network the batched AlphaZero search
evaluates once per simulation).

Reference: /root/reference/lzero/model/alphazero_model.py:14-190 (``AlphaZeroModel``,
``compute_policy_value`` = softmax(logits), value) and ``PredictionNetwork`` :193-330;
``RepresentationNetwork`` lzero/model/common.py:370-460 with ``downsample=False`` (conv3x3 without
bias, BN, ReLU, then residual blocks). DI-engine's ``ResBlock(res_type='basic', bias=False)`` is
restated from its known structure (conv3x3-BN-act, conv3x3-BN, + identity, act) and its ``MLP`` by
``model_mlp.mlp`` with LayerNorm. TicTacToe config: observation (3, 3, 3), 9 actions, 1 residual
block, 16 channels, value / policy head width 8 (zoo/board_games/tictactoe/config/
tictactoe_alphazero_sp_mode_config.py:46-54). DI-engine is absent, so outputs are not pinned to the
reference (architecture, widths, init and forward order are).
"""
from typing import Sequence

import torch
import torch.nn as nn

from .model_mlp import mlp


class ResBlock(nn.Module):
    def __init__(self, channels: int, activation: nn.Module):
        super().__init__()
        self.conv1 = nn.Conv2d(channels, channels, 3, 1, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(channels)
        self.conv2 = nn.Conv2d(channels, channels, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(channels)
        self.act = activation

    def forward(self, x):
        y = self.act(self.bn1(self.conv1(x)))
        y = self.bn2(self.conv2(y))
        return self.act(y + x)


class AlphaZeroModel(nn.Module):
    def __init__(self, observation_shape: Sequence[int] = (3, 3, 3), action_space_size: int = 9,
                 num_res_blocks: int = 1, num_channels: int = 16, value_head_channels: int = 16,
                 policy_head_channels: int = 16, fc_value_layers: Sequence[int] = (8,),
                 fc_policy_layers: Sequence[int] = (8,), value_support_size: int = 1,
                 last_linear_layer_init_zero: bool = True):
        super().__init__()
        act = nn.ReLU(inplace=True)
        C, H, W = observation_shape
        self.conv = nn.Conv2d(C, num_channels, 3, 1, 1, bias=False)
        self.norm = nn.BatchNorm2d(num_channels)
        self.rep_blocks = nn.ModuleList([ResBlock(num_channels, act) for _ in range(num_res_blocks)])
        self.pred_blocks = nn.ModuleList([ResBlock(num_channels, act) for _ in range(num_res_blocks)])
        self.conv1x1_value = nn.Conv2d(num_channels, value_head_channels, 1)
        self.conv1x1_policy = nn.Conv2d(num_channels, policy_head_channels, 1)
        self.norm_value = nn.BatchNorm2d(value_head_channels)
        self.norm_policy = nn.BatchNorm2d(policy_head_channels)
        self.flat_v, self.flat_p = value_head_channels * H * W, policy_head_channels * H * W
        self.fc_value_head = mlp(self.flat_v, fc_value_layers[0], value_support_size, len(fc_value_layers) + 1, act,
                                 'LN', output_activation=False, output_norm=False,
                                 last_linear_layer_init_zero=last_linear_layer_init_zero)
        self.fc_policy_head = mlp(self.flat_p, fc_policy_layers[0], action_space_size, len(fc_policy_layers) + 1,
                                  act, 'LN', output_activation=False, output_norm=False,
                                  last_linear_layer_init_zero=last_linear_layer_init_zero)
        self.act = act

    def forward(self, state_batch):
        x = self.act(self.norm(self.conv(state_batch)))
        for blk in self.rep_blocks:
            x = blk(x)
        for blk in self.pred_blocks:
            x = blk(x)
        v = self.act(self.norm_value(self.conv1x1_value(x))).reshape(-1, self.flat_v)
        p = self.act(self.norm_policy(self.conv1x1_policy(x))).reshape(-1, self.flat_p)
        return self.fc_policy_head(p), self.fc_value_head(v)

    def compute_policy_value(self, state_batch):
        logit, value = self.forward(state_batch)
        return torch.softmax(logit, dim=-1), value


def tictactoe_alphazero_model(random_heads: bool = True) -> AlphaZeroModel:
    """The TicTacToe config's network in eval mode; random_heads re-initialises the zero-init last
    layers so an untrained net still gives a non-uniform search."""
    m = AlphaZeroModel(last_linear_layer_init_zero=not random_heads)
    return m.eval()
