"""Collect and eval modes of LightZero's MuZeroPolicy / EfficientZeroPolicy over the GPU search.

`MuZeroCollectPolicy` is the object `MuZeroCollector` drives as `policy.collect_mode`
(DI-engine's Policy is absent): `forward(data, action_mask, temperature, to_play, epsilon,
ready_env_id)`, `reset(env_id)`, `get_attribute('cfg')`. `forward` restates
MuZeroPolicy._forward_collect (lzero/policy/muzero.py:617-740) step for step with the same host
random streams — Dirichlet root noise from `np.random.dirichlet` (:674-677) and the action from
`np.random.choice` over visits^(1/T) (`select_action`, lzero/policy/utils.py:515-539) — so the
numpy draws are the reference's on the same seed; the search itself is the drop-in
`MuZeroMCTSCtree` on the GPU (fused one-launch search for MuZeroModelMLP and the conv MuZeroModel).
This is the collector's host-parity mode; the device collector (lightzero_amd.collector) is the fast
mode with Philox streams.

`EfficientZeroCollectPolicy` restates EfficientZeroPolicy._forward_collect
(lzero/policy/efficientzero.py:538-656): the roots are prepared with the value-prefix roots and the
search gets the initial inference's reward_hidden_state roots (the LSTM (c, h), zeros at the root:
efficientzero_model.py:199-233) through the drop-in `EfficientZeroMCTSCtree`.

`eval_mode.forward(data, action_mask, to_play, ready_env_id)` on either restates _forward_eval
(muzero.py:783-867; efficientzero.py:690-770): prepare_no_noise, the search, and the argmax action
(select_action with deterministic=True) — no random draw at all.

`record = True` keeps, per forward, what a host restatement needs to replay the step exactly
(root logits and values, noises, the search's traverse seeds and per-simulation network outputs):
`records` (tests/test_gpu_muzero_collector.py replays them through the oracle).
"""
import copy

import numpy as np
import torch
from scipy.stats import entropy

from .mcts_ctree import EfficientZeroMCTSCtree, MuZeroMCTSCtree
from .scaling_transform import InverseScalarTransform
from .utils import EasyDict

# the MuZeroPolicy defaults the collect path reads (policy/muzero.py:36-228)
COLLECT_DEFAULTS = dict(
    model=dict(model_type='mlp', support_scale=300, categorical_distribution=True, frame_stack_num=1,
               action_space_size=2, observation_shape=4, image_channel=1),
    device='cuda', mcts_ctree=True, collect_with_pure_policy=False, root_dirichlet_alpha=0.3,
    root_noise_weight=0.25, num_simulations=50, discount_factor=0.997, eps=dict(eps_greedy_exploration_in_collect=False),
    game_segment_length=200, num_unroll_steps=5, td_steps=5, use_priority=False, ignore_done=False,
    gray_scale=False, transform2string=False, sampled_algo=False, gumbel_algo=False,
    use_ture_chance_label_in_chance_encoder=False, n_episode=8, type='muzero',
)


def policy_config(**overrides):
    """MuZeroPolicy-style config: COLLECT_DEFAULTS with nested overrides (EasyDict)."""
    def merge(a, b):
        for k, v in b.items():
            a[k] = merge(dict(a[k]), v) if isinstance(v, dict) and isinstance(a.get(k), dict) else v
        return a
    return EasyDict(merge(copy.deepcopy(COLLECT_DEFAULTS), overrides))


def select_action(visit_counts, temperature: float = 1, deterministic: bool = True):
    """policy/utils.py:515-539: probabilities visits^(1/T) / sum (Python floats), argmax or one
    np.random.choice draw; returns (position, entropy of the probabilities in bits)"""
    probs = [v ** (1 / temperature) for v in visit_counts]
    total = sum(probs)
    probs = [x / total for x in probs]
    pos = np.argmax(list(visit_counts)) if deterministic else np.random.choice(len(visit_counts), p=probs)
    return pos, entropy(probs, base=2)


class _EvalMode:
    """policy.eval_mode: forward = _forward_eval"""

    def __init__(self, policy):
        self._policy = policy

    def forward(self, data, action_mask=None, to_play=(-1,), ready_env_id=None):
        return self._policy.forward_eval(data, action_mask, to_play, ready_env_id)

    def reset(self, data_id=None, **kwargs):
        return None

    def get_attribute(self, name):
        return self._policy.get_attribute(name)


class MuZeroCollectPolicy:
    mcts_cls = MuZeroMCTSCtree

    def __init__(self, cfg, model):
        self._cfg = cfg
        self._model = model
        self._collect_model = model
        self._eval_model = model
        self._mcts_collect = self.mcts_cls(cfg)
        self._mcts_eval = self.mcts_cls(cfg)
        self.inverse_scalar_transform_handle = InverseScalarTransform(
            cfg.model.support_scale, cfg.device, cfg.model.categorical_distribution)
        self._collect_mcts_temperature = 1.
        self.collect_epsilon = 0.0
        self.record = False
        self.records = []

    # -- the collect_mode / eval_mode surface
    @property
    def collect_mode(self):
        return self

    @property
    def eval_mode(self):
        return _EvalMode(self)

    def get_attribute(self, name):
        return self._cfg if name == 'cfg' else getattr(self, '_' + name)

    def reset(self, data_id=None, **kwargs):
        """MuZeroPolicy keeps no per-env collect state (conv_context models aside)"""
        return None

    # -- family hooks (MuZero; EfficientZeroCollectPolicy overrides)
    def _unpack(self, out):
        """mz_network_output_unpack: (latent roots, reward roots as a list, value logits, policy logits,
        reward hidden state or None)"""
        reward_roots = out.reward
        if torch.is_tensor(reward_roots):
            reward_roots = reward_roots.detach().float().cpu().numpy().reshape(-1).tolist()
        return out.latent_state, reward_roots, out.value, out.policy_logits, None

    def _search(self, mcts, roots, latent, hidden, to_play):
        mcts.search(roots, self._collect_model, latent, to_play)

    def _roots(self, n, legal_actions):
        return self.mcts_cls.roots(n, legal_actions)

    def forward_eval(self, data, action_mask, to_play=(-1,), ready_env_id=None):
        """_forward_eval (muzero.py:783-867): no exploration noise, argmax action"""
        self._eval_model.eval()
        n = data.shape[0]
        if ready_env_id is None:
            ready_env_id = np.arange(n)
        output = {i: None for i in ready_env_id}
        with torch.no_grad():
            out = self._eval_model.initial_inference(data)
            latent, reward_roots, value, logits, hidden = self._unpack(out)
            pred_values = self.inverse_scalar_transform_handle(value).detach().cpu().numpy()
            policy_logits = logits.detach().cpu().numpy().tolist()
            legal_actions = [[i for i, x in enumerate(action_mask[j]) if x == 1] for j in range(n)]
            rec = None
            if self.record:
                rec = dict(mode='eval', data=data.detach().cpu().numpy(),
                           root_logits=np.asarray(policy_logits, np.float32), pred_values=pred_values.copy(),
                           legal=legal_actions, to_play=list(to_play), reward_roots=list(reward_roots))
                self.records.append(rec)
            roots = self._roots(n, legal_actions)
            roots.prepare_no_noise(reward_roots, policy_logits, list(to_play))
            self._mcts_eval.record = self.record
            self._search(self._mcts_eval, roots, latent, hidden, list(to_play))
            dists = roots.get_distributions()
            values = roots.get_values()
            if rec is not None:
                rec.update(search=self._mcts_eval.last_record.numpy(), dist=dists, values=values)
            for i, env_id in enumerate(ready_env_id):
                d, v = dists[i], values[i]
                pos, ent = select_action(d, temperature=1, deterministic=True)
                output[env_id] = {'action': np.where(action_mask[i] == 1.0)[0][pos], 'visit_count_distributions': d,
                                  'visit_count_distribution_entropy': ent, 'searched_value': v,
                                  'predicted_value': pred_values[i], 'predicted_policy_logits': policy_logits[i]}
            roots.clear()
        return output

    def forward(self, data, action_mask=None, temperature: float = 1, to_play=(-1,), epsilon: float = 0.25,
                ready_env_id=None):
        cfg = self._cfg
        self._collect_model.eval()
        self._collect_mcts_temperature = temperature
        self.collect_epsilon = epsilon
        n = data.shape[0]
        if ready_env_id is None:
            ready_env_id = np.arange(n)
        output = {i: None for i in ready_env_id}
        with torch.no_grad():
            out = self._collect_model.initial_inference(data)
            latent, reward_roots, value, logits, hidden = self._unpack(out)
            pred_values = self.inverse_scalar_transform_handle(value).detach().cpu().numpy()
            policy_logits = logits.detach().cpu().numpy().tolist()
            legal_actions = [[i for i, x in enumerate(action_mask[j]) if x == 1] for j in range(n)]
            rec = None
            if self.record:
                rec = dict(data=data.detach().cpu().numpy(), root_logits=np.asarray(policy_logits, np.float32),
                           pred_values=pred_values.copy(), legal=legal_actions, to_play=list(to_play),
                           reward_roots=list(reward_roots))
                self.records.append(rec)
            if cfg.collect_with_pure_policy:
                for i, env_id in enumerate(ready_env_id):
                    pv = torch.softmax(torch.tensor([policy_logits[i][a] for a in legal_actions[i]]), dim=0).tolist()
                    pv = pv / np.sum(pv)
                    idx = np.random.choice(len(legal_actions[i]), p=pv)
                    output[env_id] = {'action': np.where(action_mask[i] == 1.0)[0][idx], 'searched_value': pred_values[i],
                                      'predicted_value': pred_values[i], 'predicted_policy_logits': policy_logits[i]}
                return output
            noises = [np.random.dirichlet([cfg.root_dirichlet_alpha] * int(sum(action_mask[j]))).astype(np.float32)
                      .tolist() for j in range(n)]
            roots = self._roots(n, legal_actions)
            roots.prepare(cfg.root_noise_weight, noises, reward_roots, policy_logits, list(to_play))
            self._mcts_collect.record = self.record
            self._search(self._mcts_collect, roots, latent, hidden, list(to_play))
            dists = roots.get_distributions()
            values = roots.get_values()
            if rec is not None:
                rec.update(noises=noises, search=self._mcts_collect.last_record.numpy(), dist=dists, values=values)
            eps_greedy = cfg.eps.eps_greedy_exploration_in_collect
            for i, env_id in enumerate(ready_env_id):
                d, v = dists[i], values[i]
                pos, ent = select_action(d, temperature=self._collect_mcts_temperature, deterministic=eps_greedy)
                action = np.where(action_mask[i] == 1.0)[0][pos]
                if eps_greedy and np.random.rand() < self.collect_epsilon:
                    action = np.random.choice(legal_actions[i])
                output[env_id] = {'action': action, 'visit_count_distributions': d,
                                  'visit_count_distribution_entropy': ent, 'searched_value': v,
                                  'predicted_value': pred_values[i], 'predicted_policy_logits': policy_logits[i]}
            roots.clear()
        return output


class EfficientZeroCollectPolicy(MuZeroCollectPolicy):
    """EfficientZeroPolicy._forward_collect / _forward_eval (efficientzero.py:538-656, :690-770): roots
    prepared with the value-prefix roots, the search handed the initial inference's
    reward_hidden_state roots (ez_network_output_unpack)."""
    mcts_cls = EfficientZeroMCTSCtree

    def __init__(self, cfg, model):
        if 'lstm_horizon_len' not in cfg:  # EfficientZeroPolicy's default (efficientzero.py config)
            cfg = EasyDict(dict(cfg, lstm_horizon_len=5))
        super().__init__(cfg, model)

    def _unpack(self, out):
        vp = out.value_prefix
        if torch.is_tensor(vp):
            vp = vp.detach().float().cpu().numpy().reshape(-1).tolist()
        return out.latent_state, vp, out.value, out.policy_logits, out.reward_hidden_state

    def _search(self, mcts, roots, latent, hidden, to_play):
        mcts.search(roots, self._collect_model, latent, hidden, to_play)
