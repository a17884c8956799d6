"""GameSegment — the trajectory block the collector hands to the replay buffer.

Same surface and field semantics as /root/reference/lzero/mcts/buffer/game_segment.py:10-334
(``reset``, ``append``, ``store_search_stats``, ``pad_over``, ``is_full``,
``game_segment_to_array``, ``get_obs``, ``get_unroll_obs``, ``zero_obs``, ``legal_actions``,
``__len__``), so `MuZeroGameBuffer.push_game_segments` consumes it unchanged. DI-engine is absent:
the config is any attribute-style object with the fields the reference reads
(num_unroll_steps, td_steps, discount_factor, gray_scale, transform2string, sampled_algo,
gumbel_algo, use_ture_chance_label_in_chance_encoder, model.{frame_stack_num,
action_space_size, observation_shape, image_channel}). ``transform2string`` needs DI-engine's
jpeg helpers and raises here.

``from_arrays`` (not in the reference) builds a finished, array-form segment in one go from
device-recorded episode arrays — what the device collector uses instead of a per-step append
loop (lightzero_amd.worker.muzero_collector).
"""
import copy
from typing import List

import numpy as np


class GameSegment:

    def __init__(self, action_space, game_segment_length: int = 200, config=None) -> None:
        self.action_space = action_space
        self.game_segment_length = game_segment_length
        self.num_unroll_steps = config.num_unroll_steps
        self.td_steps = config.td_steps
        self.frame_stack_num = config.model.frame_stack_num
        self.discount_factor = config.discount_factor
        self.action_space_size = config.model.action_space_size
        self.gray_scale = config.get("gray_scale", False)
        self.transform2string = config.get("transform2string", False)
        self.sampled_algo = config.get("sampled_algo", False)
        self.gumbel_algo = config.get("gumbel_algo", False)
        self.use_ture_chance_label_in_chance_encoder = config.get("use_ture_chance_label_in_chance_encoder", False)
        if self.transform2string:
            raise NotImplementedError("transform2string needs DI-engine's jpeg helpers (not installed)")
        shape = config.model.observation_shape
        if isinstance(shape, int) or len(shape) == 1:
            self.zero_obs_shape = shape
        else:  # image observations [C, H, W]
            self.zero_obs_shape = (config.model.image_channel, shape[-2], shape[-1])
        self._clear()
        self.target_values, self.target_rewards, self.target_policies = [], [], []

    def _clear(self):
        self.obs_segment, self.action_segment, self.reward_segment = [], [], []
        self.child_visit_segment, self.root_value_segment = [], []
        self.action_mask_segment, self.to_play_segment = [], []
        self.improved_policy_probs = []
        if self.sampled_algo:
            self.root_sampled_actions = []
        if self.use_ture_chance_label_in_chance_encoder:
            self.chance_segment = []

    # -- reading
    def get_unroll_obs(self, timestep: int, num_unroll_steps: int = 0, padding: bool = False):
        """o[t : t + frame_stack_num + num_unroll_steps], padded with the last frame if asked"""
        obs = self.obs_segment[timestep:timestep + self.frame_stack_num + num_unroll_steps]
        if padding:
            short = self.frame_stack_num + num_unroll_steps - len(obs)
            if short > 0:
                obs = np.concatenate((obs, np.array([obs[-1]] * short)))
        return obs

    def zero_obs(self) -> List:
        return [np.zeros(self.zero_obs_shape, dtype=np.float32) for _ in range(self.frame_stack_num)]

    def get_obs(self) -> List:
        """the stacked observation the policy sees now: the frame_stack_num frames ending at the
        latest one (obs entries lead rewards by frame_stack_num)"""
        t = len(self.reward_segment)
        assert len(self.obs_segment) - self.frame_stack_num == t, \
            f"timestep_obs: {len(self.obs_segment) - self.frame_stack_num}, timestep_reward: {t}"
        return self.obs_segment[t:t + self.frame_stack_num]

    def get_targets(self, timestep: int):
        return self.target_values[timestep], self.target_rewards[timestep], self.target_policies[timestep]

    def legal_actions(self):
        return list(range(self.action_space.n))

    def is_full(self) -> bool:
        return len(self.action_segment) >= self.game_segment_length

    def __len__(self):
        return len(self.action_segment)

    # -- writing
    def reset(self, init_observations) -> None:
        """start the segment from the frame_stack_num frames of the observation window"""
        self._clear()
        assert len(init_observations) == self.frame_stack_num
        self.obs_segment.extend(copy.deepcopy(o) for o in init_observations)

    def append(self, action, obs, reward, action_mask=None, to_play: int = -1, chance: int = 0) -> None:
        """transition (a_t, o_{t+1}, r_t, action_mask_t, to_play_t)"""
        self.action_segment.append(action)
        self.obs_segment.append(obs)
        self.reward_segment.append(reward)
        self.action_mask_segment.append(action_mask)
        self.to_play_segment.append(to_play)
        if self.use_ture_chance_label_in_chance_encoder:
            self.chance_segment.append(chance)

    def store_search_stats(self, visit_counts: List, root_value, root_sampled_actions: List = None,
                           improved_policy: List = None, idx: int = None) -> None:
        """root visit distribution (visit / sum, sum 0 -> 1e-6) and searched root value"""
        total = sum(visit_counts)
        if total == 0:
            total = 1e-6
        dist = [v / total for v in visit_counts]
        if idx is not None:
            self.child_visit_segment[idx] = dist
            self.root_value_segment[idx] = root_value
            self.improved_policy_probs[idx] = improved_policy
            return
        self.child_visit_segment.append(dist)
        self.root_value_segment.append(root_value)
        if self.sampled_algo:
            self.root_sampled_actions.append(root_sampled_actions)
        if self.gumbel_algo:
            self.improved_policy_probs.append(improved_policy)

    def pad_over(self, next_segment_observations: List, next_segment_rewards: List, next_segment_root_values: List,
                 next_segment_child_visits: List, next_segment_improved_policy: List = None,
                 next_chances: List = None) -> None:
        """append the next block's first frames / rewards / root values / visit distributions, so the
        bootstrapped targets at the end of this block are computable (game_segment.py:151-196)"""
        U, TD = self.num_unroll_steps, self.td_steps
        assert len(next_segment_observations) <= U
        assert len(next_segment_child_visits) <= U
        assert len(next_segment_root_values) <= U + TD
        assert len(next_segment_rewards) <= U + TD - 1
        if self.gumbel_algo:
            assert len(next_segment_improved_policy) <= U + TD
        self.obs_segment.extend(copy.deepcopy(o) for o in next_segment_observations)
        self.reward_segment.extend(next_segment_rewards)
        self.root_value_segment.extend(next_segment_root_values)
        self.child_visit_segment.extend(next_segment_child_visits)
        if self.gumbel_algo:
            self.improved_policy_probs.extend(next_segment_improved_policy)
        if self.use_ture_chance_label_in_chance_encoder:
            self.chance_segment.extend(next_chances)

    def game_segment_to_array(self) -> None:
        """lists -> numpy arrays (child visits as an object array when their lengths differ)"""
        self.obs_segment = np.array(self.obs_segment)
        self.action_segment = np.array(self.action_segment)
        self.reward_segment = np.array(self.reward_segment)
        cv = self.child_visit_segment
        ragged = any(len(x) != len(cv[0]) for x in cv) if len(cv) else False
        self.child_visit_segment = np.array(cv, dtype=object) if ragged else np.array(cv)
        self.root_value_segment = np.array(self.root_value_segment)
        self.improved_policy_probs = np.array(self.improved_policy_probs)
        self.action_mask_segment = np.array(self.action_mask_segment)
        self.to_play_segment = np.array(self.to_play_segment)
        if self.use_ture_chance_label_in_chance_encoder:
            self.chance_segment = np.array(self.chance_segment)

    @classmethod
    def from_arrays(cls, action_space, game_segment_length, config, obs, action, reward, child_visits, root_value,
                    action_mask, to_play):
        """A finished segment in array form, as game_segment_to_array leaves it (fields already cut
        and padded by the caller; lightzero_amd.worker.segments)."""
        g = cls(action_space, game_segment_length, config)
        g.obs_segment, g.action_segment, g.reward_segment = obs, action, reward
        g.child_visit_segment, g.root_value_segment = child_visits, root_value
        g.improved_policy_probs = np.array([])
        g.action_mask_segment, g.to_play_segment = action_mask, to_play
        return g
