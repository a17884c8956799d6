"""MuZeroCollector — LightZero's self-play collector surface over the GPU search.

Constructor, `collect`, `reset`, `reset_env`, `reset_policy`, `envstep`, `close` and the return
value are those of /root/reference/lzero/worker/muzero_collector.py:18-719 (registered there as
'episode_muzero'):

    MuZeroCollector(collect_print_freq, env, policy, tb_logger, exp_name, instance_name, policy_config)
    collect(n_episode=None, train_iter=0, policy_kwargs={'temperature', 'epsilon'},
            collect_with_pure_policy=False)
      -> ([GameSegment, ...], [{'priorities', 'done', 'unroll_plus_td_steps'}, ...])

Two paths behind the one surface:

- host loop (any BaseEnvManager-like `env`, any collect-mode `policy`): the reference's loop
  (:399-705) — ready-env bookkeeping with `remain_episode`, policy forward on the stacked
  observations, env step, store_search_stats / append, `game_segment_length` rollover with
  `pad_over` of the previous segment (:229-301, :566-591), end-of-episode saves (:612-632),
  `_compute_priorities` (:200-227). With `lightzero_amd.policy.MuZeroCollectPolicy` the search runs
  on the GPU and the noise / action draws come from numpy exactly as the reference draws them: the
  collector's host-parity mode.
- device path (`env` a `lightzero_amd.envs.DeviceEnvManager` — CartPole or the Breakout stand-in —, `policy` a
  MuZeroCollectPolicy): every env steps inside one HIP graph per iteration
  (lightzero_amd.collector.DeviceCollector: fused search, action selection, CartPole physics and
  recording on the GPU, Philox streams), the host polls finished episodes, replays the reference's
  ready-env / remain_episode schedule on their lengths and cuts the counted episodes into the same
  segments, flags, priorities and pool order (lightzero_amd.worker.segments).

DI-engine is absent: logging goes to the `logging` module (and `tb_logger.add_scalar` when one is
given), rank / world size and the statistics all-reduce come from torch.distributed.
"""
import logging
import time
from collections import deque

import numpy as np
import torch
import torch.distributed as dist
from scipy.stats import entropy

from ..envs import DeviceEnvManager
from ..game_segment import GameSegment
from .segments import EpisodeSchedule, episode_segments


def _rank():
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def _world_size():
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def _allreduce_sum(x):
    """ding.utils.allreduce_data(x, 'sum') over the default group"""
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor(float(x), dtype=torch.float64, device=dev)
    dist.all_reduce(t)
    return t.item()


def _to_ndarray(x):
    """ding.torch_utils.to_ndarray for the values an env observation holds"""
    if isinstance(x, np.ndarray):
        return x
    if torch.is_tensor(x):
        return x.cpu().numpy()
    if isinstance(x, (bool, str)) or x is None:
        return x
    return np.array(x)


def _stack_observation(frames, model_type):
    """lzero.mcts.utils.prepare_observation: [B, S, O] -> [B, S*O] (mlp), [B, S, C, W, H] ->
    [B, S*C, W, H] (conv)"""
    a = np.array(frames)
    B = a.shape[0]
    if model_type in ('mlp', 'mlp_context'):
        if a.ndim != 3:
            raise ValueError("For 'mlp' model_type, the observation must have 3 dimensions [B, S, O]")
        return a.reshape(B, -1)
    if a.ndim == 3:
        return a[..., np.newaxis]
    if a.ndim == 5:
        return a.reshape(B, a.shape[1] * a.shape[2], a.shape[3], a.shape[4])
    return a


class _Timer:
    """the slice of DI-engine's EasyTimer the collector uses (`with timer:`, `.value`)"""

    def __init__(self):
        self.value = 0.0

    def __enter__(self):
        self._t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        self.value = time.perf_counter() - self._t0
        return False


class MuZeroCollector:
    config = dict()

    def __init__(self, collect_print_freq: int = 100, env=None, policy=None, tb_logger=None,
                 exp_name: str = 'default_experiment', instance_name: str = 'collector', policy_config=None) -> None:
        self._exp_name = exp_name
        self._instance_name = instance_name
        self._collect_print_freq = collect_print_freq
        self._timer = _Timer()
        self._end_flag = False
        self._rank = _rank()
        self._world_size = _world_size()
        self._logger = logging.getLogger(f"lightzero_amd.{exp_name}.{instance_name}")
        self._tb_logger = tb_logger if self._rank == 0 else None
        self.policy_config = policy_config
        self.collect_with_pure_policy = policy_config.collect_with_pure_policy
        self._device = None  # the DeviceCollector of the device path, built on first use
        self.reset(policy, env)

    # ------------------------------------------------------------------ lifecycle (:87-195)
    def reset_env(self, _env=None) -> None:
        if _env is not None:
            self._env = _env
            self._env.launch()
            self._env_num = self._env.env_num
            self._device = None
        else:
            self._env.reset()

    def reset_policy(self, _policy=None) -> None:
        assert hasattr(self, '_env'), "please set env first"
        if _policy is not None:
            self._policy = _policy
            self._default_n_episode = _policy.get_attribute('cfg').get('n_episode', None)
            self._device = None
        self._policy.reset()

    def reset(self, _policy=None, _env=None) -> None:
        if _env is not None:
            self.reset_env(_env)
        if _policy is not None:
            self.reset_policy(_policy)
        self._env_info = {env_id: {'time': 0., 'step': 0} for env_id in range(self._env_num)}
        self._episode_info = []
        self._total_envstep_count = 0
        self._total_episode_count = 0
        self._total_duration = 0
        self._last_train_iter = 0
        self._end_flag = False
        self.game_segment_pool = deque(maxlen=int(1e6))
        self.unroll_plus_td_steps = self.policy_config.num_unroll_steps + self.policy_config.td_steps

    def _reset_stat(self, env_id: int) -> None:
        self._env_info[env_id] = {'time': 0., 'step': 0}

    @property
    def envstep(self) -> int:
        return self._total_envstep_count

    def close(self) -> None:
        if self._end_flag:
            return
        self._end_flag = True
        self._env.close()
        if self._tb_logger:
            self._tb_logger.flush()
            self._tb_logger.close()

    def __del__(self) -> None:
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------ segments (:200-301)
    def _compute_priorities(self, i, pred_values_lst, search_values_lst):
        """L1 distance between predicted and searched root values (+1e-6), or None (max priority)"""
        if not self.policy_config.use_priority:
            return None
        pred = torch.from_numpy(np.array(pred_values_lst[i])).float().view(-1)
        search = torch.from_numpy(np.array(search_values_lst[i])).float().view(-1)
        return torch.nn.L1Loss(reduction='none')(pred, search).numpy() + 1e-6

    def pad_and_save_last_trajectory(self, i, last_game_segments, last_game_priorities, game_segments, done) -> None:
        """pad segment i's previous block with the current block's leading entries and save it"""
        cfg = self.policy_config
        fs, U = cfg.model.frame_stack_num, cfg.num_unroll_steps
        cur = game_segments[i]
        pad_obs = cur.obs_segment[fs:fs + U]
        pad_child_visits = cur.child_visit_segment[:U]
        pad_rewards = cur.reward_segment[:self.unroll_plus_td_steps - 1]
        pad_root_values = cur.root_value_segment[:self.unroll_plus_td_steps]
        kw = {}
        if cfg.gumbel_algo:
            kw['next_segment_improved_policy'] = cur.improved_policy_probs[:self.unroll_plus_td_steps]
        if cfg.use_ture_chance_label_in_chance_encoder:
            kw['next_chances'] = cur.chance_segment[:self.unroll_plus_td_steps - 1]
        last_game_segments[i].pad_over(pad_obs, pad_rewards, pad_root_values, pad_child_visits, **kw)
        last_game_segments[i].game_segment_to_array()
        self.game_segment_pool.append((last_game_segments[i], last_game_priorities[i], done[i]))
        last_game_segments[i] = None
        last_game_priorities[i] = None

    def _new_segment(self):
        return GameSegment(self._env.action_space, game_segment_length=self.policy_config.game_segment_length,
                           config=self.policy_config)

    def _return_pool(self):
        segs = [s for s, _, _ in self.game_segment_pool]
        meta = [{'priorities': p, 'done': d, 'unroll_plus_td_steps': self.unroll_plus_td_steps}
                for _, p, d in self.game_segment_pool]
        self.game_segment_pool.clear()
        return segs, meta

    # ------------------------------------------------------------------ collect (:305-719)
    def collect(self, n_episode=None, train_iter: int = 0, policy_kwargs=None, collect_with_pure_policy: bool = False):
        if n_episode is None:
            if self._default_n_episode is None:
                raise RuntimeError("Please specify collect n_episode")
            n_episode = self._default_n_episode
        if n_episode < self._env_num:
            raise AssertionError(f"collect: n_episode ({n_episode}) must be at least the env count ({self._env_num})")
        policy_kwargs = {} if policy_kwargs is None else policy_kwargs
        temperature = policy_kwargs['temperature']
        epsilon = policy_kwargs['epsilon']
        if self._device_path(collect_with_pure_policy):
            return_data, collected_step, collected_episode = self._collect_device(n_episode, temperature)
        else:
            return_data, collected_step, collected_episode = self._collect_host(n_episode, temperature, epsilon,
                                                                                collect_with_pure_policy)
        collected_duration = sum(d['time'] for d in self._episode_info)
        if self._world_size > 1:
            collected_step = _allreduce_sum(collected_step)
            collected_episode = _allreduce_sum(collected_episode)
            collected_duration = _allreduce_sum(collected_duration)
        self._total_envstep_count += collected_step
        self._total_episode_count += collected_episode
        self._total_duration += collected_duration
        self._output_log(train_iter)
        return return_data

    def _collect_host(self, n_episode, temperature, epsilon, collect_with_pure_policy):
        cfg = self.policy_config
        fs = cfg.model.frame_stack_num
        env_nums = self._env_num
        init_obs = self._wait_ready()
        action_mask_dict = {i: _to_ndarray(init_obs[i]['action_mask']) for i in range(env_nums)}
        to_play_dict = {i: _to_ndarray(init_obs[i]['to_play']) for i in range(env_nums)}
        chance_dict = {i: _to_ndarray(init_obs[i]['chance']) for i in range(env_nums)} \
            if cfg.use_ture_chance_label_in_chance_encoder else None
        game_segments = [self._new_segment() for _ in range(env_nums)]
        windows = []
        for env_id in range(env_nums):
            windows.append(deque([_to_ndarray(init_obs[env_id]['observation']) for _ in range(fs)], maxlen=fs))
            game_segments[env_id].reset(windows[env_id])
        dones = np.array([False for _ in range(env_nums)])
        last_game_segments = [None] * env_nums
        last_game_priorities = [None] * env_nums
        search_values_lst = [[] for _ in range(env_nums)]
        pred_values_lst = [[] for _ in range(env_nums)]
        eps_steps_lst, visit_entropies_lst = np.zeros(env_nums), np.zeros(env_nums)
        collected_episode = collected_step = 0
        ready_env_id = set()
        remain_episode = n_episode
        pure_visits = [0.0] * self._env.action_space.n if collect_with_pure_policy else None
        while True:
            with self._timer:
                obs = self._env.ready_obs
                new_available = set(obs.keys()).difference(ready_env_id)
                ready_env_id = ready_env_id.union(set(list(new_available)[:remain_episode]))
                remain_episode -= min(len(new_available), remain_episode)
                stack_obs = [game_segments[env_id].get_obs() for env_id in ready_env_id]
                action_mask_dict = {env_id: action_mask_dict[env_id] for env_id in ready_env_id}
                to_play_dict = {env_id: to_play_dict[env_id] for env_id in ready_env_id}
                action_mask = [action_mask_dict[env_id] for env_id in ready_env_id]
                to_play = [to_play_dict[env_id] for env_id in ready_env_id]
                if chance_dict is not None:
                    chance_dict = {env_id: chance_dict[env_id] for env_id in ready_env_id}
                data = torch.from_numpy(_stack_observation([_to_ndarray(o) for o in stack_obs], cfg.model.model_type))
                data = data.to(cfg.device)
                policy_output = self._policy.forward(data, action_mask, temperature, to_play, epsilon,
                                                     ready_env_id=ready_env_id)
                actions = {k: v['action'] for k, v in policy_output.items()}
                timesteps = self._env.step({env_id: actions[env_id] for env_id in ready_env_id})
            interaction_duration = self._timer.value / len(timesteps)
            for env_id, timestep in timesteps.items():
                with self._timer:
                    if timestep.info.get('abnormal', False):
                        self._env.reset({env_id: None})
                        self._policy.reset([env_id])
                        self._reset_stat(env_id)
                        self._logger.info(f"env {env_id}: abnormal step, reset ({timestep.info})")
                        continue
                    out = policy_output[env_id]
                    obs_t, reward, done = timestep.obs, timestep.reward, timestep.done
                    seg = game_segments[env_id]
                    if collect_with_pure_policy:
                        seg.store_search_stats(pure_visits, 0)
                    else:
                        seg.store_search_stats(out['visit_count_distributions'], out['searched_value'])
                    if chance_dict is not None:
                        seg.append(actions[env_id], _to_ndarray(obs_t['observation']), reward, action_mask_dict[env_id],
                                   to_play_dict[env_id], chance_dict[env_id])
                    else:
                        seg.append(actions[env_id], _to_ndarray(obs_t['observation']), reward, action_mask_dict[env_id],
                                   to_play_dict[env_id])
                    # the next action's mask / player come with this observation
                    action_mask_dict[env_id] = _to_ndarray(obs_t['action_mask'])
                    to_play_dict[env_id] = _to_ndarray(obs_t['to_play'])
                    if chance_dict is not None:
                        chance_dict[env_id] = _to_ndarray(obs_t['chance'])
                    dones[env_id] = False if cfg.ignore_done else done
                    if not collect_with_pure_policy:
                        visit_entropies_lst[env_id] += out['visit_count_distribution_entropy']
                    eps_steps_lst[env_id] += 1
                    if cfg.use_priority:
                        pred_values_lst[env_id].append(out['predicted_value'])
                        search_values_lst[env_id].append(out['searched_value'])
                    windows[env_id].append(_to_ndarray(obs_t['observation']))
                    if seg.is_full():  # rollover: pad + save the previous block, this one becomes it
                        if last_game_segments[env_id] is not None:
                            self.pad_and_save_last_trajectory(env_id, last_game_segments, last_game_priorities,
                                                              game_segments, dones)
                        priorities = self._compute_priorities(env_id, pred_values_lst, search_values_lst)
                        pred_values_lst[env_id] = []
                        search_values_lst[env_id] = []
                        last_game_segments[env_id] = seg
                        last_game_priorities[env_id] = priorities
                        game_segments[env_id] = self._new_segment()
                        game_segments[env_id].reset(windows[env_id])
                    self._env_info[env_id]['step'] += 1
                    collected_step += 1
                self._env_info[env_id]['time'] += self._timer.value + interaction_duration
                if not timestep.done:
                    continue
                info = {'reward': timestep.info['eval_episode_return'], 'time': self._env_info[env_id]['time'],
                        'step': self._env_info[env_id]['step']}
                if not collect_with_pure_policy:
                    info['visit_entropy'] = visit_entropies_lst[env_id] / eps_steps_lst[env_id]
                collected_episode += 1
                self._episode_info.append(info)
                if last_game_segments[env_id] is not None:
                    self.pad_and_save_last_trajectory(env_id, last_game_segments, last_game_priorities, game_segments,
                                                      dones)
                priorities = self._compute_priorities(env_id, pred_values_lst, search_values_lst)
                game_segments[env_id].game_segment_to_array()
                if len(game_segments[env_id].reward_segment) != 0:
                    self.game_segment_pool.append((game_segments[env_id], priorities, dones[env_id]))
                if n_episode > self._env_num:
                    init_obs = self._wait_ready()
                    new_available = set(init_obs.keys()).difference(ready_env_id)
                    ready_env_id = ready_env_id.union(set(list(new_available)[:remain_episode]))
                    remain_episode -= min(len(new_available), remain_episode)
                    action_mask_dict[env_id] = _to_ndarray(init_obs[env_id]['action_mask'])
                    to_play_dict[env_id] = _to_ndarray(init_obs[env_id]['to_play'])
                    if chance_dict is not None:
                        chance_dict[env_id] = _to_ndarray(init_obs[env_id]['chance'])
                    game_segments[env_id] = self._new_segment()
                    windows[env_id] = deque([init_obs[env_id]['observation'] for _ in range(fs)], maxlen=fs)
                    game_segments[env_id].reset(windows[env_id])
                    last_game_segments[env_id] = None
                    last_game_priorities[env_id] = None
                pred_values_lst[env_id] = []
                search_values_lst[env_id] = []
                eps_steps_lst[env_id] = 0
                visit_entropies_lst[env_id] = 0
                self._policy.reset([env_id])
                self._reset_stat(env_id)
                ready_env_id.remove(env_id)
            if collected_episode >= n_episode:
                return self._return_pool(), collected_step, collected_episode

    def _wait_ready(self):
        """every env's reset observation (subprocess managers may lag behind, :341-351)"""
        obs = self._env.ready_obs
        while len(obs.keys()) != self._env_num:
            time.sleep(0.001)
            obs = self._env.ready_obs
        return obs

    # ------------------------------------------------------------------ device path
    def _device_path(self, collect_with_pure_policy):
        from ..policy import MuZeroCollectPolicy
        cfg = self.policy_config
        # MuZero and EfficientZero policies (EfficientZeroCollectPolicy subclasses MuZeroCollectPolicy): the
        # device collector's search step picks the EfficientZero search (value-prefix roots, the reward LSTM)
        # from the model, as EfficientZeroPolicy._forward_collect does (efficientzero.py:538-656)
        return (isinstance(self._env, DeviceEnvManager) and isinstance(self._policy, MuZeroCollectPolicy)
                and not collect_with_pure_policy and not cfg.eps.eps_greedy_exploration_in_collect
                and cfg.model.frame_stack_num == self._env.frame_stack)

    def _device_collector(self, temperature):
        from ..collector import DeviceCollector
        cfg = self.policy_config
        if self._device is None:
            env = self._env
            self._device = DeviceCollector(
                self._policy._model, env.env_num, cfg.num_simulations, device=cfg.device,
                max_episode_steps=env.max_episode_steps, episode_slots=cfg.get('device_episode_slots', 8),
                temperature=temperature, noise_alpha=cfg.root_dirichlet_alpha, noise_weight=cfg.root_noise_weight,
                seed=env.seed, rng_mode=cfg.get('device_rng', 'glibc'), graph=True,
                poll_every=cfg.get('device_poll_every', 4), record_pred=bool(cfg.use_priority),
                support_scale=cfg.model.support_scale, env=env.env_kind,
                categorical_distribution=bool(cfg.model.get('categorical_distribution', True)),
                search_cfg=dict(discount_factor=float(cfg.get('discount_factor', 0.997)),
                                lstm_horizon_len=int(cfg.get('lstm_horizon_len', 5))))
        else:
            self._device.set_temperature(temperature)
        return self._device

    def _collect_device(self, n_episode, temperature):
        """All envs step together on the device; the reference's schedule decides which episodes
        count: every env starts one, and each finished one hands the env a new episode while
        `remain_episode` lasts (ascending env ids within an iteration, as the reference's ready-set
        union does). Episodes an env plays beyond its share (it would sit idle in the reference)
        are dropped. Segments are cut per counted episode and saved in the reference's pool order."""
        cfg = self.policy_config
        n = self._env_num
        col = self._device_collector(temperature)
        col.restart()
        sched = EpisodeSchedule(n, n_episode)
        pool = []
        infos = []
        collected_step = 0
        mask = np.ones(col.A, np.int8)
        t_start = time.perf_counter()
        while not sched.complete:
            for _ in range(col.poll_every):
                col.step()
            finished = col.pull_new()
            for start, i, e in sched.take([(e["env_id"], len(e["action_segment"]), e) for e in finished]):
                L = len(e["action_segment"])
                for it, k, seg, prio, d in episode_segments(cfg, self._env.action_space, e["obs_segment"],
                                                            e["action_segment"], e["reward_segment"], e["visits"],
                                                            e["root_value_segment"], e.get("pred_value_segment"),
                                                            start, mask, -1):
                    pool.append((it, i, k, seg, prio, d))
                collected_step += L
                # the env's eval_episode_return (muzero_collector.py:596-603): the unclipped game score
                # for Atari, the reward sum for CartPole (recorded on the device, lzm_*_collect_step)
                infos.append({'reward': float(e["episode_return"]), 'time': 0.0, 'step': L,
                              'visit_entropy': self._visit_entropy(e["visits"], temperature)})
        # the loop's wall time is the collect duration (all envs step together on the device); each
        # counted episode gets the share of it its steps make up, so the per-episode times sum to it
        wall = time.perf_counter() - t_start
        for d in infos:
            d['time'] = wall * d['step'] / max(collected_step, 1)
        self._episode_info.extend(infos)
        self.last_schedule = sched  # (tests: the counted episodes per env)
        pool.sort(key=lambda x: (x[0], x[1], x[2]))
        for _, _, _, seg, prio, d in pool:
            self.game_segment_pool.append((seg, prio, d))
        return self._return_pool(), collected_step, sched.collected

    @staticmethod
    def _visit_entropy(visits, temperature):
        """mean over the episode's steps of select_action's entropy of visits^(1/T) / sum, in bits"""
        p = visits.astype(np.float64) ** (1.0 / temperature)
        p = p / p.sum(axis=1, keepdims=True)
        return float(np.mean([entropy(row, base=2) for row in p]))

    # ------------------------------------------------------------------ logs (:721-769)
    def _output_log(self, train_iter: int) -> None:
        if self._rank != 0:
            return
        if (train_iter - self._last_train_iter) < self._collect_print_freq or not self._episode_info:
            return
        self._last_train_iter = train_iter
        eps = self._episode_info
        envstep_count = sum(d['step'] for d in eps)
        duration = sum(d['time'] for d in eps)
        rewards = [d['reward'] for d in eps]
        ent = [d['visit_entropy'] for d in eps] if not self.collect_with_pure_policy else [0.0]
        self._total_duration += duration
        info = {
            'episode_count': len(eps), 'envstep_count': envstep_count,
            'avg_envstep_per_episode': envstep_count / len(eps),
            'avg_envstep_per_sec': envstep_count / duration if duration > 0 else float('inf'),
            'avg_episode_per_sec': len(eps) / duration if duration > 0 else float('inf'),
            'collect_time': duration, 'reward_mean': np.mean(rewards), 'reward_std': np.std(rewards),
            'reward_max': np.max(rewards), 'reward_min': np.min(rewards),
            'total_envstep_count': self._total_envstep_count, 'total_episode_count': self._total_episode_count,
            'total_duration': self._total_duration, 'visit_entropy': np.mean(ent),
        }
        self._episode_info.clear()
        self._logger.info("collect end:\n{}".format('\n'.join('{}: {}'.format(k, v) for k, v in info.items())))
        if self._tb_logger is not None:
            for k, v in info.items():
                self._tb_logger.add_scalar('{}_iter/'.format(self._instance_name) + k, v, train_iter)
                if k != 'total_envstep_count':
                    self._tb_logger.add_scalar('{}_step/'.format(self._instance_name) + k, v,
                                               self._total_envstep_count)
