"""Trajectory return across ranks: the only data-path collective of the sharded
collector.

Each rank's DeviceCollector records its envs' episodes in device-resident slots: one recorded frame
per step (rec_frames [n, E, T+1, *frame_shape] — CartPole's float32 [4] observation, or an Atari env's
u8 [1, 64, 64] grey frame; GameSegment stores one frame per step and stacks frame_stack_num of them for
the model, lzero/mcts/buffer/game_segment.py:95-149), rec_action / rec_reward / rec_value [n, E, T],
rec_visits [n, E, T, A]. After `collect()`, the finished episodes are packed on the device into a
`TrajBlock` (no host copy of the payload), flattened into ONE byte buffer per rank, and returned over the
process group (RCCL over xGMI on the GPU node, gloo in the CPU tests) either to the learner rank alone
(`gather_packed`: each rank sends its buffer once, point to point) or to every rank (`all_gather_packed`:
one all-gather), and unpacked into GameSegment-shaped dicts (the fields of game_segment.py:229-294) only
when a caller asks for them. The
collector statistics are sum-reduced as MuZeroCollector does under DDP
(lzero/worker/muzero_collector.py:709-712).

TrajBlock layout, episode j of length L occupying L + 1 consecutive rows:
  frames  [rows, *frame_shape] (the recorded dtype: u8 frames stay u8 on the wire) — o_0 .. o_L;
  scalars [rows, W] float32, W = 3 + A (+ 1 with predicted values) — [action_t | reward_t |
          root visit counts_t (A) | root_value_t (| pred_value_t)]; row L (the obs segment has L + 1
          entries, the others L) is zero but for its reward column, which holds the episode's return
          (the env's eval_episode_return, muzero_collector.py:596-603 — for Atari the UNCLIPPED score,
          while reward_t is clipped);
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
                  rec_pred=None, frame_scale: float = 1.0, ep_return=None) -> TrajBlock:
    """episodes: [(env_id, slot, L)] -> TrajBlock on the buffers' device (torch ops; the device
    collector packs with the lzm_episodes_* kernels, same layout). ep_return [n, E] (optional): the
    slots' episode returns, written to each episode's row L."""
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
    if ep_return is not None:
        lt = torch.from_numpy(last).to(dev)
        sc[lt, 1] = ep_return[i_t[lt], e_t[lt]].to(torch.float32)
    return TrajBlock(frames, sc, torch.from_numpy(index), frame_scale)


def unpack_episodes(block: TrajBlock, A: int, rank: int = 0) -> List[dict]:
    """GameSegment-shaped dicts from one rank's block (host arrays). obs_segment holds the L + 1
    observations as the reference stores them (float32, frame * frame_scale); child_visit_segment is
    store_search_stats' visit / sum in float64; `visits` keeps the raw counts; `episode_return` is the
    env's eval_episode_return (row L's reward column)."""
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
                 action_mask_segment=np.ones((L, A), np.int8), episode_return=float(sc[L, 1]))
        if has_pred:
            e["pred_value_segment"] = sc[:L, 3 + A].copy()
        eps.append(e)
    return eps


def _align(n: int, a: int = 16) -> int:
    return (int(n) + a - 1) // a * a


def _flat_layout(rows: int, n_ep: int, frame_bytes: int, W: int):
    """byte offsets of (frames, scalars, index) in a block's flat wire buffer and its total length: the
    three arrays back to back, each part starting on a 16-byte boundary"""
    f, sc, ix = rows * frame_bytes, rows * W * 4, n_ep * 24
    o_s = _align(f)
    o_i = o_s + _align(sc)
    return 0, o_s, o_i, o_i + ix


def _frame_bytes(block: TrajBlock) -> int:
    f = block.frames
    return int(np.prod(tuple(f.shape[1:]), dtype=np.int64)) * (f.element_size() if torch.is_tensor(f) else f.itemsize)


def flatten_block(block: TrajBlock, device=None) -> torch.Tensor:
    """ONE uint8 buffer holding the block's frames, scalars and index (the layout of _flat_layout): what a
    rank puts on the wire — a single collective or send per rank instead of one per array."""
    dev = torch.device(device) if device is not None else block.scalars.device
    W = block.scalars.shape[1]
    o_f, o_s, o_i, n = _flat_layout(block.rows, block.num_episodes, _frame_bytes(block), W)
    buf = torch.zeros(n, dtype=torch.uint8, device=dev)
    if block.rows:
        buf[o_f:o_f + block.rows * _frame_bytes(block)] = block.frames.contiguous().reshape(-1).view(torch.uint8).to(dev)
        buf[o_s:o_s + block.rows * W * 4] = block.scalars.contiguous().reshape(-1).view(torch.uint8).to(dev)
    if block.num_episodes:
        buf[o_i:n] = block.index.to(torch.int64).contiguous().reshape(-1).view(torch.uint8).to(dev)
    return buf


def unflatten_block(buf: torch.Tensor, rows: int, n_ep: int, frame_shape, frame_dtype, W: int,
                    frame_scale: float) -> TrajBlock:
    """the TrajBlock a flat wire buffer holds (views into `buf`, no copy)"""
    fb = int(np.prod(tuple(frame_shape), dtype=np.int64)) * torch.empty((), dtype=frame_dtype).element_size()
    o_f, o_s, o_i, n = _flat_layout(rows, n_ep, fb, W)
    frames = buf[o_f:o_f + rows * fb].view(frame_dtype).reshape((rows,) + tuple(frame_shape))
    scalars = buf[o_s:o_s + rows * W * 4].view(torch.float32).reshape(rows, W)
    index = buf[o_i:n].view(torch.int64).reshape(n_ep, 3)
    return TrajBlock(frames, scalars, index, frame_scale)


def _wire_device(block: TrajBlock, group):
    dev = block.scalars.device
    if dev.type == "cuda" and dist.get_backend(group) == "gloo":
        return torch.device("cpu")  # gloo moves host tensors only (RCCL groups keep them on the GPU)
    return dev


def _exchange_sizes(block: TrajBlock, dev, group):
    """(rows, episodes) of every rank's block: one all-gather of 16 bytes per rank"""
    world = dist.get_world_size(group)
    sizes = torch.tensor([block.rows, block.num_episodes], dtype=torch.int64, device=dev)
    all_sizes = [torch.zeros_like(sizes) for _ in range(world)]
    dist.all_gather(all_sizes, sizes, group=group)
    return [tuple(int(v) for v in s.cpu().tolist()) for s in all_sizes]


def all_gather_packed(block: TrajBlock, group=None, to_host: bool = True) -> List[TrajBlock]:
    """All-gather variable-size TrajBlocks: one size exchange, then ONE all-gather of every rank's flat
    wire buffer (frames in their own dtype — u8 frames travel as bytes —, scalars and index back to back,
    padded to the largest rank's length) on the payload's device (RCCL for GPU tensors). Returns every
    rank's block in rank order — host numpy arrays, or device tensors with to_host=False (views into the
    received buffers)."""
    world = dist.get_world_size(group)
    dev = _wire_device(block, group)
    all_sizes = _exchange_sizes(block, dev, group)
    fshape, fdtype, W = tuple(block.frames.shape[1:]), block.frames.dtype, block.scalars.shape[1]
    fb = _frame_bytes(block)
    lens = [_flat_layout(r, e, fb, W)[3] for r, e in all_sizes]
    flat = flatten_block(block, dev)
    padded = torch.zeros(max(1, max(lens)), dtype=torch.uint8, device=dev)
    padded[:flat.numel()] = flat
    recv = [torch.empty_like(padded) for _ in range(world)]
    dist.all_gather(recv, padded, group=group)
    out = []
    for r, (nr, ne) in enumerate(all_sizes):
        blk = unflatten_block(recv[r], nr, ne, fshape, fdtype, W, block.frame_scale)
        out.append(blk.numpy() if to_host else blk)
    return out


def gather_packed(block: TrajBlock, dst: int = 0, group=None, to_host: bool = True) -> List[TrajBlock]:
    """Gather-to-learner: only rank `dst` receives. One size exchange, then each other rank
    sends its flat wire buffer ONCE, at its exact length, point to point (RCCL send / recv over xGMI on the
    GPU node; batch_isend_irecv). Rank dst returns every rank's block in rank order (its own without a copy);
    the other ranks return []. Bytes moved per collect: the sum of the non-learner payloads, received by
    the learner alone (the all-gather moves world - 1 padded payloads to EVERY rank)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = _wire_device(block, group)
    all_sizes = _exchange_sizes(block, dev, group)
    fshape, fdtype, W = tuple(block.frames.shape[1:]), block.frames.dtype, block.scalars.shape[1]
    fb = _frame_bytes(block)
    lens = [_flat_layout(r, e, fb, W)[3] for r, e in all_sizes]
    peer = (lambda r: r) if group is None else (lambda r: dist.get_global_rank(group, r))
    ops, bufs = [], {}
    if rank == dst:
        for r in range(world):
            if r != dst and lens[r]:
                bufs[r] = torch.empty(lens[r], dtype=torch.uint8, device=dev)
                ops.append(dist.P2POp(dist.irecv, bufs[r], peer(r), group))
    elif lens[rank]:
        ops.append(dist.P2POp(dist.isend, flatten_block(block, dev), peer(dst), group))
    for w in (dist.batch_isend_irecv(ops) if ops else []):
        w.wait()
    if rank != dst:
        return []
    out = []
    for r, (nr, ne) in enumerate(all_sizes):
        if r == dst:
            blk = block
        elif lens[r]:
            blk = unflatten_block(bufs[r], nr, ne, fshape, fdtype, W, block.frame_scale)
        else:
            blk = unflatten_block(torch.zeros(0, dtype=torch.uint8, device=dev), 0, 0, fshape, fdtype, W,
                                  block.frame_scale)
        out.append(blk.numpy() if to_host else blk)
    return out


def wire_bytes(block: TrajBlock) -> int:
    """length of the block's flat wire buffer"""
    return _flat_layout(block.rows, block.num_episodes, _frame_bytes(block), block.scalars.shape[1])[3]


def allreduce_stats(collected_step: float, collected_episode: float, collected_duration: float, device,
                    group=None):
    """muzero_collector.py:709-712: sum the three collector statistics over ranks."""
    if torch.device(device).type == "cuda" and dist.get_backend(group) == "gloo":
        device = "cpu"
    t = torch.tensor([collected_step, collected_episode, collected_duration], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return tuple(float(v) for v in t.cpu().tolist())
