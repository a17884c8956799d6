"""Reanalyze: policy targets from a fresh search over replay positions.

Restates the search part of MuZeroGameBuffer._compute_target_policy_reanalyzed
(lzero/mcts/buffer/game_buffer_muzero.py:519-660) on device tensors: initial_inference over the
transition batch (batch_size x (num_unroll_steps + 1) positions, 1,536 at the reference's CartPole
defaults), roots prepared with or without root noise (`reanalyze_noise`), one MuZeroMCTSCtree.search
(the fused kernel for MuZeroModelMLP), then per position `visits / sum(visits)` scattered onto the
legal action indices, zeros where `policy_mask` is 0. The legal lists are built from the action mask
on the device (Roots.from_action_mask) and the scatter index is that device table, so the call
makes no host round trip. The list bookkeeping around it (game segment indices, child_visit
write-back) stays with the replay buffer (out of scope).
"""
import torch

from .mcts_ctree import MuZeroMCTSCtree
from .utils import EasyDict


def reanalyze_policy_targets(model, obs, action_mask, policy_mask, cfg, to_play=None, noises=None,
                             noise_weight=0.25, mini_infer_size=None, seeds=None):
    """obs [N, ...] float, action_mask [N, A] {0,1}, policy_mask [N] {0,1} (device tensors).

    cfg: num_simulations, discount_factor, model.support_scale, pb_c_base / pb_c_init /
    value_delta_max (MuZeroMCTSCtree defaults otherwise). noises [N, A] (Dirichlet, legal order)
    or None for prepare_no_noise. Returns (target_policies [N, A], root_values [N]) on the device.
    """
    dev = obs.device
    N = obs.shape[0]
    A = action_mask.shape[1]
    mcfg = MuZeroMCTSCtree.default_config()
    mcfg.update(cfg)
    mcfg.device = dev
    mcts = MuZeroMCTSCtree(EasyDict(mcfg))
    with torch.no_grad():
        step = mini_infer_size or N
        outs = [model.initial_inference(obs[i:i + step]) for i in range(0, N, step)]
        latent = torch.cat([o.latent_state for o in outs])
        logits = torch.cat([o.policy_logits for o in outs])
        rewards = torch.zeros(N, dtype=torch.float32, device=dev)  # MuZero initial reward is 0
        tp = (torch.full((N,), -1, dtype=torch.int32, device=dev) if to_play is None
              else to_play.to(device=dev, dtype=torch.int32))
        # legal lists from the mask on the device (the reference builds them on the host)
        roots = MuZeroMCTSCtree.roots_from_mask(action_mask.to(dev))
        legal_dev = roots._legal_dev[0]
        roots.prepare_device(noise_weight if noises is not None else 0.0,
                             noises if noises is not None else None, rewards, logits, tp)
        mcts.search(roots, model, latent, tp, seeds=seeds)
        t = roots.tree
        dist = t.distributions().to(torch.float32)  # [N, A] in legal order, -1 padded
        values = t.values()
        roots.clear()
        valid = dist >= 0
        vis = torch.where(valid, dist, torch.zeros_like(dist))
        probs = vis / vis.sum(dim=1, keepdim=True).clamp_min(1.0)
        # scatter legal-order probabilities onto action indices (the device legal lists, -1 padded)
        idx = legal_dev.to(torch.int64)
        target = torch.zeros((N, A), dtype=torch.float32, device=dev)
        # padded slots add 0 at index 0 (scatter_add: no write conflicts)
        target.scatter_add_(1, idx.clamp_min(0), torch.where(idx >= 0, probs, torch.zeros_like(probs)))
        target = target * policy_mask.to(dev, torch.float32).unsqueeze(1)
    return target, values
