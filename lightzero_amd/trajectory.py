"""Trajectory return across ranks: the only data-path collective of the sharded
collector.

Each rank's DeviceCollector records its envs' episodes in device-resident slots: one recorded frame
per step (rec_frames [n, E, T+1, *frame_shape] — CartPole's float32 [4] observation, or an Atari env's
u8 [1, 64, 64] grey frame; GameSegment stores one frame per step and stacks frame_stack_num of them for
the model, lzero/mcts/buffer/game_segment.py:95-149), rec_action / rec_reward / rec_value [n, E, T],
rec_visits [n, E, T, A]. After `collect()`, the finished episodes are packed on the device into a
`TrajBlock` (no host copy of the payload), the blocks of all ranks are exchanged with all-gathers over
the process group (RCCL over xGMI on the GPU node, gloo in the CPU tests), and unpacked into
GameSegment-shaped dicts (the fields of game_segment.py:229-294) only when a caller asks for them. The
collector statistics are sum-reduced as MuZeroCollector does under DDP
(lzero/worker/muzero_collector.py:709-712).

TrajBlock layout, episode j of length L occupying L + 1 consecutive rows:
  frames  [rows, *frame_shape] (the recorded dtype: u8 frames stay u8 on the wire) — o_0 .. o_L;
  scalars [rows, W] float32, W = 3 + A (+ 1 with predicted values) — [action_t | reward_t |
          root visit counts_t (A) | root_value_t (| pred_value_t)], row L zeros (the obs segment has
          L + 1 entries, the others L);
  index   [n_ep, 3] int64 — (env_id, L, first row).
Actions and visit counts are small integers, exact in float32. `frame_scale` maps a stored frame to
the observation the reference's GameSegment holds (1 / 255 for u8 grey frames: the wrappers'
ScaledFloatFrame; 1 for float observations).
"""
from dataclasses import dataclass
from typing import List, Tuple, Union

import numpy as np
import torch
import torch.distributed as dist


def scalar_width(A: int, pred: bool = False) -> int:
    return 3 + A + int(bool(pred))


@dataclass
class TrajBlock:
    frames: Union[torch.Tensor, np.ndarray]
    scalars: Union[torch.Tensor, np.ndarray]
    index: Union[torch.Tensor, np.ndarray]
    frame_scale: float = 1.0

    @property
    def num_episodes(self) -> int:
        return int(self.index.shape[0])

    @property
    def rows(self) -> int:
        return int(self.scalars.shape[0])

    @property
    def nbytes(self) -> int:
        return sum(int(x.numel() * x.element_size()) if torch.is_tensor(x) else int(x.nbytes)
                   for x in (self.frames, self.scalars, self.index))

    def numpy(self) -> "TrajBlock":
        f = (lambda x: x.cpu().numpy()) if torch.is_tensor(self.scalars) else (lambda x: x)
        return TrajBlock(f(self.frames), f(self.scalars), f(self.index), self.frame_scale)


def pack_episodes(rec_frames, rec_action, rec_reward, rec_visits, rec_value, episodes: List[Tuple[int, int, int]],
                  rec_pred=None, frame_scale: float = 1.0) -> TrajBlock:
    """episodes: [(env_id, slot, L)] -> TrajBlock on the buffers' device (torch ops; the device
    collector packs with the lzm_episodes_* kernels, same layout)."""
    dev = rec_frames.device
    frame_shape = tuple(rec_frames.shape[3:])
    A = rec_visits.shape[-1]
    W = scalar_width(A, rec_pred is not None)
    lens = np.array([L for _, _, L in episodes], np.int64)
    rows = int((lens + 1).sum())
    index = np.zeros((len(episodes), 3), np.int64)
    if not episodes:
        return TrajBlock(torch.zeros((0,) + frame_shape, dtype=rec_frames.dtype, device=dev),
                         torch.zeros((0, W), dtype=torch.float32, device=dev), torch.from_numpy(index), frame_scale)
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
    frames = rec_frames[i_t, e_t, t_t].contiguous()
    sc = torch.empty((rows, W), dtype=torch.float32, device=dev)
    sc[:, 0:1] = rec_action[i_t, e_t, tc].to(torch.float32).unsqueeze(1) * keep
    sc[:, 1:2] = rec_reward[i_t, e_t, tc].unsqueeze(1) * keep
    sc[:, 2:2 + A] = rec_visits[i_t, e_t, tc].to(torch.float32) * keep
    sc[:, 2 + A:3 + A] = rec_value[i_t, e_t, tc].unsqueeze(1) * keep
    if rec_pred is not None:
        sc[:, 3 + A:] = rec_pred[i_t, e_t, tc].unsqueeze(1) * keep
    return TrajBlock(frames, sc, torch.from_numpy(index), frame_scale)


def unpack_episodes(block: TrajBlock, A: int, rank: int = 0) -> List[dict]:
    """GameSegment-shaped dicts from one rank's block (host arrays). obs_segment holds the L + 1
    observations as the reference stores them (float32, frame * frame_scale); child_visit_segment is
    store_search_stats' visit / sum in float64; `visits` keeps the raw counts."""
    b = block.numpy()
    eps = []
    has_pred = b.scalars.shape[1] == scalar_width(A, True)
    for env_id, L, r0 in np.asarray(b.index, np.int64):
        sc = b.scalars[r0:r0 + L + 1]
        fr = b.frames[r0:r0 + L + 1]
        obs = fr.astype(np.float32) * np.float32(b.frame_scale) if b.frame_scale != 1.0 else fr.astype(np.float32)
        visits = np.rint(sc[:L, 2:2 + A]).astype(np.int64)
        tot = visits.sum(axis=1, keepdims=True).astype(np.float64)
        tot[tot == 0] = 1e-6
        e = dict(rank=rank, env_id=int(env_id), obs_segment=obs, action_segment=np.rint(sc[:L, 0]).astype(np.int64),
                 reward_segment=sc[:L, 1].copy(), visits=visits, child_visit_segment=visits / tot,
                 root_value_segment=sc[:L, 2 + A].copy(), to_play_segment=np.full(L, -1, np.int32),
                 action_mask_segment=np.ones((L, A), np.int8))
        if has_pred:
            e["pred_value_segment"] = sc[:L, 3 + A].copy()
        eps.append(e)
    return eps


def all_gather_packed(block: TrajBlock, group=None, to_host: bool = True) -> List[TrajBlock]:
    """All-gather variable-size TrajBlocks: one size exchange, then one padded all-gather each of the
    frames (in their own dtype: u8 frames travel as bytes), the scalars and the index (on the payload's
    device: RCCL for GPU tensors). Returns every rank's block in rank order — host numpy arrays, or
    device tensors with to_host=False (what a learner on the same GPU consumes)."""
    world = dist.get_world_size(group)
    dev = block.scalars.device
    if dev.type == "cuda" and dist.get_backend(group) == "gloo":
        dev = torch.device("cpu")  # gloo all-gathers host tensors only (RCCL groups keep them on the GPU)
    frame_shape = tuple(block.frames.shape[1:])
    W = block.scalars.shape[1]
    sizes = torch.tensor([block.rows, block.num_episodes], dtype=torch.int64, device=dev)
    all_sizes = [torch.zeros_like(sizes) for _ in range(world)]
    dist.all_gather(all_sizes, sizes, group=group)
    all_sizes = [s.cpu().tolist() for s in all_sizes]
    max_rows = max(1, max(s[0] for s in all_sizes))
    max_eps = max(1, max(s[1] for s in all_sizes))

    def padded(x, n, shape, dtype):
        out = torch.zeros((n,) + shape, dtype=dtype, device=dev)
        out[:x.shape[0]] = x.to(dev)
        return out

    parts = [padded(block.frames, max_rows, frame_shape, block.frames.dtype),
             padded(block.scalars, max_rows, (W,), torch.float32),
             padded(block.index, max_eps, (3,), torch.int64)]
    gathered = []
    for x in parts:
        lst = [torch.empty_like(x) for _ in range(world)]
        dist.all_gather(lst, x, group=group)
        gathered.append(lst)
    out = []
    for r, (nr, ne) in enumerate(all_sizes):
        blk = TrajBlock(gathered[0][r][:nr], gathered[1][r][:nr], gathered[2][r][:ne], block.frame_scale)
        out.append(blk.numpy() if to_host else blk)
    return out


def allreduce_stats(collected_step: float, collected_episode: float, collected_duration: float, device,
                    group=None):
    """muzero_collector.py:709-712: sum the three collector statistics over ranks."""
    if torch.device(device).type == "cuda" and dist.get_backend(group) == "gloo":
        device = "cpu"
    t = torch.tensor([collected_step, collected_episode, collected_duration], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return tuple(float(v) for v in t.cpu().tolist())
