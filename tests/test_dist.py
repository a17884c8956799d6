"""Multi-process (gloo, world_size 2, CPU) coverage of the sharded path.

The search shards by envs: each rank owns its envs' trees and seeds and nothing crosses ranks in
the data path; the only collective is bench.py's max-reduce of the elapsed time. These tests run
the same shard layout as bench.py (bench.shard_seed) with the oracle search on each rank and check
  1. every rank's shard result equals a single-process run of that shard (no cross-rank state),
  2. bench.slowest_rank_seconds reduces to the max over ranks and bench.whole_job_rate counts all
     ranks' simulations.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import bench
from tests.helpers import run_scripted_search_oracle

B_SHARD, S, A = 12, 12, 3


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rec = run_scripted_search_oracle(B_SHARD, S, A, seed=bench.shard_seed(rank), players=1 + rank % 2)
        mine = torch.from_numpy(rec["dist"].astype(np.int64))
        gathered = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(gathered, mine)
        el = bench.slowest_rank_seconds(0.5 + rank, world, torch.device("cpu"))
        if rank == 0:
            np.savez(os.path.join(out_dir, "r0.npz"), dist=torch.stack(gathered).numpy(), el=el,
                     rate=bench.whole_job_rate(B_SHARD, S, 3, world, el))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 4])
def test_env_sharded_search_gloo(tmp_path, world):
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    r = np.load(tmp_path / "r0.npz")
    for rank in range(world):
        ref = run_scripted_search_oracle(B_SHARD, S, A, seed=bench.shard_seed(rank), players=1 + rank % 2)
        assert np.array_equal(r["dist"][rank], ref["dist"]), f"rank {rank} shard differs from a solo run"
        assert (r["dist"][rank].sum(axis=1) == S).all()
    assert float(r["el"]) == world - 0.5  # max over ranks (0.5, 1.5, ...)
    assert float(r["rate"]) == world * B_SHARD * S * 3 / (world - 0.5)


def test_single_rank_helpers():
    assert bench.slowest_rank_seconds(2.0, 1, torch.device("cpu")) == 2.0
    assert bench.whole_job_rate(256, 50, 20, 1, 1.0) == 256 * 50 * 20
    assert bench.shard_seed(0) != bench.shard_seed(1)


# ---------------------------------------------------------------- trajectory all-gather (§8(e))
N_ENV, E_SLOTS, T_MAX, ACT = 5, 3, 9, 2
# CartPole: one float32 [4] observation per step; Atari (config 5): one u8 [1, 64, 64] grey frame per step
KINDS = {"vector": ((4,), torch.float32, 1.0), "image": ((1, 64, 64), torch.uint8, 1.0 / 255.0)}


def _fake_records(rank, kind="vector"):
    """a rank's collector slots with random contents and a rank-dependent set of finished episodes"""
    shape, dtype, _ = KINDS[kind]
    g = torch.Generator().manual_seed(100 + rank)
    if dtype == torch.uint8:
        frames = torch.randint(0, 256, (N_ENV, E_SLOTS, T_MAX + 1) + shape, generator=g, dtype=torch.uint8)
    else:
        frames = torch.randn((N_ENV, E_SLOTS, T_MAX + 1) + shape, generator=g)
    rec = dict(obs=frames,
               action=torch.randint(0, ACT, (N_ENV, E_SLOTS, T_MAX), generator=g, dtype=torch.int32),
               reward=torch.randn(N_ENV, E_SLOTS, T_MAX, generator=g),
               child=torch.randint(0, 30, (N_ENV, E_SLOTS, T_MAX, ACT), generator=g, dtype=torch.int32),
               value=torch.randn(N_ENV, E_SLOTS, T_MAX, generator=g))
    rng = np.random.default_rng(rank)
    eps = [(int(i), int(e), int(rng.integers(1, T_MAX + 1))) for i in range(N_ENV) for e in range(E_SLOTS)
           if rng.random() < 0.5 + 0.3 * rank]
    return rec, eps


def _expected(rank, kind="vector"):
    rec, eps = _fake_records(rank, kind)
    scale = KINDS[kind][2]
    out = []
    for i, e, L in eps:
        obs = rec["obs"][i, e, :L + 1].numpy().astype(np.float32)
        out.append(dict(env_id=i, obs=obs * np.float32(scale) if scale != 1.0 else obs,
                        action=rec["action"][i, e, :L].numpy(), reward=rec["reward"][i, e, :L].numpy(),
                        child=rec["child"][i, e, :L].numpy(), value=rec["value"][i, e, :L].numpy()))
    return out


def _check_episodes(got, want, rank):
    assert len(got) == len(want)
    for g, w in zip(got, want):
        assert g["rank"] == rank and g["env_id"] == w["env_id"]
        assert g["obs_segment"].dtype == np.float32 and np.array_equal(g["obs_segment"], w["obs"])
        assert np.array_equal(g["action_segment"], w["action"].astype(np.int64))
        assert np.array_equal(g["reward_segment"], w["reward"])
        assert np.array_equal(g["visits"], w["child"].astype(np.int64))
        tot = w["child"].sum(axis=1, keepdims=True).astype(np.float64)
        tot[tot == 0] = 1e-6
        assert np.array_equal(g["child_visit_segment"], w["child"] / tot)  # store_search_stats, float64
        assert np.array_equal(g["root_value_segment"], w["value"])
        assert g["to_play_segment"].shape == (len(w["action"]),)


def _pack(rank, kind):
    from lightzero_amd.trajectory import pack_episodes
    rec, eps = _fake_records(rank, kind)
    return pack_episodes(rec["obs"], rec["action"], rec["reward"], rec["child"], rec["value"], eps,
                         frame_scale=KINDS[kind][2]), eps


def _traj_worker(rank, world, port, out_dir, kind, mode="all_gather"):
    from lightzero_amd.trajectory import all_gather_packed, allreduce_stats, gather_packed
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        block, eps = _pack(rank, kind)
        if mode == "all_gather":
            blocks = all_gather_packed(block)
        else:  # gather-to-learner: rank 0 alone receives
            blocks = gather_packed(block, dst=0)
            assert (len(blocks) == world) if rank == 0 else (blocks == [])
            if rank == 0:
                assert blocks[0] is not None and blocks[0].rows == block.rows
        stats = allreduce_stats(10.0 * (rank + 1), float(len(eps)), 0.25, torch.device("cpu"))
        arrays = {}
        for r, b in enumerate(blocks):
            arrays.update({f"f{r}": b.frames, f"s{r}": b.scalars, f"i{r}": b.index, f"c{r}": np.float64(b.frame_scale)})
        np.savez(os.path.join(out_dir, f"r{rank}.npz"), stats=np.array(stats), **arrays)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("mode", ["all_gather", "gather"])
@pytest.mark.parametrize("kind", ["vector", "image"])
def test_trajectory_return_gloo_world2(tmp_path, kind, mode):
    """all_gather: every rank ends with every rank's episodes; gather: the learner (rank 0) alone does —
    CartPole vectors and config 5's u8 image frames (one flat byte buffer per rank on the wire, unpacked
    to the reference's float32 frame / 255); the statistics are summed on every rank"""
    world = 2
    mp.spawn(_traj_worker, args=(world, _free_port(), str(tmp_path), kind, mode), nprocs=world, join=True)
    _check_gathered(tmp_path, world, kind, mode)


def _check_gathered(tmp_path, world, kind, mode):
    from lightzero_amd.trajectory import TrajBlock, unpack_episodes
    for me in range(world):
        r = np.load(tmp_path / f"r{me}.npz")
        n_eps = sum(len(_fake_records(k)[1]) for k in range(world))
        assert tuple(r["stats"]) == (10.0 * world * (world + 1) / 2, float(n_eps), 0.25 * world)
        if mode == "gather" and me != 0:
            assert "f0" not in r.files  # nothing received off the learner
            continue
        for rank in range(world):  # every receiving rank holds every rank's episodes
            blk = TrajBlock(r[f"f{rank}"], r[f"s{rank}"], r[f"i{rank}"], float(r[f"c{rank}"]))
            assert blk.frames.dtype == (np.uint8 if kind == "image" else np.float32)
            _check_episodes(unpack_episodes(blk, ACT, rank), _expected(rank, kind), rank)


@pytest.mark.parametrize("kind", ["vector", "image"])
def test_flat_wire_buffer_round_trip(kind):
    """flatten_block / unflatten_block: the block's three arrays in one 16-byte-aligned byte buffer and
    back, bit for bit (and the empty block)"""
    from lightzero_amd.trajectory import flatten_block, unflatten_block, wire_bytes
    for rank in (0, 1):
        block, _ = _pack(rank, kind)
        buf = flatten_block(block)
        assert buf.dtype == torch.uint8 and buf.numel() == wire_bytes(block)
        b2 = unflatten_block(buf, block.rows, block.num_episodes, tuple(block.frames.shape[1:]), block.frames.dtype,
                             block.scalars.shape[1], block.frame_scale)
        assert torch.equal(b2.frames, block.frames) and torch.equal(b2.scalars, block.scalars)
        assert torch.equal(b2.index, block.index.to(torch.int64))
    rec, _ = _fake_records(0, kind)
    from lightzero_amd.trajectory import pack_episodes
    b0 = pack_episodes(rec["obs"], rec["action"], rec["reward"], rec["child"], rec["value"], [])
    assert flatten_block(b0).numel() == 0


@pytest.mark.parametrize("kind", ["vector", "image"])
def test_pack_unpack_round_trip_and_empty(kind):
    from lightzero_amd.trajectory import pack_episodes, unpack_episodes
    block, eps = _pack(0, kind)
    rows = sum(L + 1 for _, _, L in eps)
    assert block.scalars.shape == (rows, 3 + ACT) and tuple(block.frames.shape) == (rows,) + KINDS[kind][0]
    _check_episodes(unpack_episodes(block, ACT), _expected(0, kind), 0)
    rec, _ = _fake_records(0, kind)
    b0 = pack_episodes(rec["obs"], rec["action"], rec["reward"], rec["child"], rec["value"], [])
    assert b0.scalars.shape == (0, 3 + ACT) and tuple(b0.index.shape) == (0, 3) and b0.frames.shape[0] == 0
    assert unpack_episodes(b0, ACT) == []


def test_image_episode_segments_frame_stack():
    """an image episode through the segment cutter: every segment starts with the frame_stack_num
    window ending at its first frame (the reset frame repeated at the episode start, game_segment.py:
    95-127) and carries one frame per step after it (muzero_collector.py:305-632)"""
    from lightzero_amd.trajectory import unpack_episodes
    from lightzero_amd.utils import EasyDict
    from lightzero_amd.worker.segments import episode_segments
    block, eps = _pack(1, "image")
    ep = max(unpack_episodes(block, ACT), key=lambda e: len(e["action_segment"]))
    L, fs = len(ep["action_segment"]), 4
    cfg = EasyDict(dict(game_segment_length=4, num_unroll_steps=2, td_steps=3, discount_factor=0.997,
                        model=EasyDict(dict(frame_stack_num=fs, action_space_size=ACT, observation_shape=(4, 64, 64),
                                            image_channel=1))))

    class Space:
        n = ACT
    segs = episode_segments(cfg, Space(), ep["obs_segment"], ep["action_segment"], ep["reward_segment"], ep["visits"],
                            ep["root_value_segment"], None, 0, np.ones(ACT, np.int8), -1)
    obs = ep["obs_segment"]
    window = np.concatenate([np.repeat(obs[:1], fs - 1, axis=0), obs])
    for j, (_, _, seg, _, _) in enumerate(segs):
        s0, n = 4 * j, len(seg.action_segment)
        assert seg.obs_segment.shape[1:] == (1, 64, 64)
        assert np.array_equal(seg.obs_segment[:fs + n], window[s0:s0 + fs + n])
        assert np.array_equal(seg.action_segment, ep["action_segment"][s0:s0 + n])
    assert sum(len(s.action_segment) for _, _, s, _, _ in segs) == L


@pytest.mark.timeout(300)
@pytest.mark.parametrize("mode", ["all_gather", "gather"])
def test_trajectory_return_gloo_world4(tmp_path, mode):
    """four ranks (the driver's 8-GPU node runs 1, 2, 4 and 8): config 5's u8 frames with ragged episode
    counts per rank, every receiving rank holding every rank's episodes in rank order"""
    world = 4
    mp.spawn(_traj_worker, args=(world, _free_port(), str(tmp_path), "image", mode), nprocs=world, join=True)
    _check_gathered(tmp_path, world, "image", mode)
