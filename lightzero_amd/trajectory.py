"""Trajectory return across ranks: the only data-path collective of the sharded
collector.

Each rank's DeviceCollector records its envs' episodes in device-resident slots (rec_obs
[n, E, T+1, obs], rec_action / rec_reward / rec_value [n, E, T], rec_visits [n, E, T, A]). After
`collect()`, the finished episodes are packed on the device into one float32 block (no host copy
of the payload), the blocks of all ranks are exchanged with one all-gather over the process group
(RCCL over xGMI on the GPU node, gloo in the CPU tests), and unpacked into GameSegment-shaped
dicts (the fields of lzero/mcts/buffer/game_segment.py:229-294). The collector statistics are
sum-reduced as MuZeroCollector does under DDP (lzero/worker/muzero_collector.py:709-712).

Packed layout: episode j of length L occupies L + 1 consecutive rows of width
W = obs_dim + 1 + 1 + A + 1 (+ 1 with predicted values): [obs_t | action_t | reward_t |
root visit counts_t (A) | root_value_t (| pred_value_t)]; row L carries the final observation (the
obs segment has L + 1 entries) and zeros elsewhere. Actions and visit counts are small integers,
exact in float32. The index is int64 [n_ep, 3] = (env_id, L, first row).
"""
from typing import List, Tuple

import numpy as np
import torch
import torch.distributed as dist


def row_width(obs_dim: int, A: int, pred: bool = False) -> int:
    return obs_dim + 3 + A + int(bool(pred))


def pack_episodes(rec_obs, rec_action, rec_reward, rec_visits, rec_value, episodes: List[Tuple[int, int, int]],
                  rec_pred=None):
    """episodes: [(env_id, slot, L)] -> (packed f32 [rows, W] on the buffers' device, index i64 [n_ep, 3])."""
    dev = rec_obs.device
    obs_dim, A = rec_obs.shape[-1], rec_visits.shape[-1]
    W = row_width(obs_dim, A, rec_pred is not None)
    lens = np.array([L for _, _, L in episodes], np.int64)
    rows = int((lens + 1).sum())
    index = np.zeros((len(episodes), 3), np.int64)
    if not episodes:
        return torch.zeros((0, W), dtype=torch.float32, device=dev), torch.from_numpy(index)
    ii = np.repeat([i for i, _, _ in episodes], lens + 1)
    ee = np.repeat([e for _, e, _ in episodes], lens + 1)
    starts = np.concatenate([[0], np.cumsum(lens + 1)[:-1]])
    tt = np.arange(rows) - np.repeat(starts, lens + 1)
    last = tt == np.repeat(lens, lens + 1)  # the final-observation row of each episode
    index[:, 0] = [i for i, _, _ in episodes]
    index[:, 1] = lens
    index[:, 2] = starts
    i_t, e_t, t_t = (torch.from_numpy(a).to(dev) for a in (ii, ee, tt))
    tc = torch.from_numpy(np.where(last, 0, tt)).to(dev)  # clamp to a valid step for the other fields
    keep = torch.from_numpy(~last).to(dev).to(torch.float32).unsqueeze(1)
    out = torch.empty((rows, W), dtype=torch.float32, device=dev)
    c = obs_dim
    out[:, :c] = rec_obs[i_t, e_t, t_t]
    out[:, c:c + 1] = rec_action[i_t, e_t, tc].to(torch.float32).unsqueeze(1) * keep
    out[:, c + 1:c + 2] = rec_reward[i_t, e_t, tc].unsqueeze(1) * keep
    out[:, c + 2:c + 2 + A] = rec_visits[i_t, e_t, tc].to(torch.float32) * keep
    out[:, c + 2 + A:c + 3 + A] = rec_value[i_t, e_t, tc].unsqueeze(1) * keep
    if rec_pred is not None:
        out[:, c + 3 + A:] = rec_pred[i_t, e_t, tc].unsqueeze(1) * keep
    return out, torch.from_numpy(index)


def unpack_episodes(packed: np.ndarray, index: np.ndarray, obs_dim: int, A: int, rank: int = 0) -> List[dict]:
    """GameSegment-shaped dicts from one rank's block (host arrays). child_visit_segment is
    store_search_stats' visit / sum in float64; `visits` keeps the raw counts."""
    eps = []
    has_pred = packed.shape[1] == row_width(obs_dim, A, True)
    c = obs_dim
    for env_id, L, r0 in np.asarray(index, np.int64):
        blk = packed[r0:r0 + L + 1]
        visits = np.rint(blk[:L, c + 2:c + 2 + A]).astype(np.int64)
        tot = visits.sum(axis=1, keepdims=True).astype(np.float64)
        tot[tot == 0] = 1e-6
        e = dict(rank=rank, env_id=int(env_id), obs_segment=blk[:, :c].copy(),
                 action_segment=np.rint(blk[:L, c]).astype(np.int64), reward_segment=blk[:L, c + 1].copy(),
                 visits=visits, child_visit_segment=visits / tot, root_value_segment=blk[:L, c + 2 + A].copy(),
                 to_play_segment=np.full(L, -1, np.int32), action_mask_segment=np.ones((L, A), np.int8))
        if has_pred:
            e["pred_value_segment"] = blk[:L, c + 3 + A].copy()
        eps.append(e)
    return eps


def all_gather_packed(packed: torch.Tensor, index: torch.Tensor, group=None):
    """All-gather variable-size (packed, index) blocks: one size exchange, then one padded
    all-gather of the payload and one of the index (on the payload's device: RCCL for GPU tensors).
    Returns host numpy [(packed_r, index_r)] for every rank r."""
    world = dist.get_world_size(group)
    dev = packed.device
    if dev.type == "cuda" and dist.get_backend(group) == "gloo":
        dev = torch.device("cpu")  # gloo all-gathers host tensors only (RCCL groups keep them on the GPU)
    W = packed.shape[1]
    sizes = torch.tensor([packed.shape[0], index.shape[0]], dtype=torch.int64, device=dev)
    all_sizes = [torch.zeros_like(sizes) for _ in range(world)]
    dist.all_gather(all_sizes, sizes, group=group)
    all_sizes = [s.cpu().tolist() for s in all_sizes]
    max_rows = max(1, max(s[0] for s in all_sizes))
    max_eps = max(1, max(s[1] for s in all_sizes))
    pay = torch.zeros((max_rows, W), dtype=torch.float32, device=dev)
    pay[:packed.shape[0]] = packed.to(dev)
    idx = torch.zeros((max_eps, 3), dtype=torch.int64, device=dev)
    idx[:index.shape[0]] = index.to(dev)
    pays = [torch.empty_like(pay) for _ in range(world)]
    idxs = [torch.empty_like(idx) for _ in range(world)]
    dist.all_gather(pays, pay, group=group)
    dist.all_gather(idxs, idx, group=group)
    return [(p[:s[0]].cpu().numpy(), i[:s[1]].cpu().numpy()) for p, i, s in zip(pays, idxs, all_sizes)]


def allreduce_stats(collected_step: float, collected_episode: float, collected_duration: float, device,
                    group=None):
    """muzero_collector.py:709-712: sum the three collector statistics over ranks."""
    if torch.device(device).type == "cuda" and dist.get_backend(group) == "gloo":
        device = "cpu"
    t = torch.tensor([collected_step, collected_episode, collected_duration], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return tuple(float(v) for v in t.cpu().tolist())
