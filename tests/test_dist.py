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
def test_env_sharded_search_gloo_world2(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    r = np.load(tmp_path / "r0.npz")
    for rank in range(world):
        ref = run_scripted_search_oracle(B_SHARD, S, A, seed=bench.shard_seed(rank), players=1 + rank % 2)
        assert np.array_equal(r["dist"][rank], ref["dist"]), f"rank {rank} shard differs from a solo run"
        assert (r["dist"][rank].sum(axis=1) == S).all()
    assert float(r["el"]) == 1.5  # max over ranks (0.5, 1.5)
    assert float(r["rate"]) == world * B_SHARD * S * 3 / 1.5


def test_single_rank_helpers():
    assert bench.slowest_rank_seconds(2.0, 1, torch.device("cpu")) == 2.0
    assert bench.whole_job_rate(256, 50, 20, 1, 1.0) == 256 * 50 * 20
    assert bench.shard_seed(0) != bench.shard_seed(1)


# ---------------------------------------------------------------- trajectory all-gather (§8(e))
N_ENV, E_SLOTS, T_MAX, OBS, ACT = 5, 3, 9, 4, 2


def _fake_records(rank):
    """a rank's collector slots with random contents and a rank-dependent set of finished episodes"""
    g = torch.Generator().manual_seed(100 + rank)
    rec = dict(obs=torch.randn(N_ENV, E_SLOTS, T_MAX + 1, OBS, generator=g),
               action=torch.randint(0, ACT, (N_ENV, E_SLOTS, T_MAX), generator=g, dtype=torch.int32),
               reward=torch.randn(N_ENV, E_SLOTS, T_MAX, generator=g),
               child=torch.randint(0, 30, (N_ENV, E_SLOTS, T_MAX, ACT), generator=g, dtype=torch.int32),
               value=torch.randn(N_ENV, E_SLOTS, T_MAX, generator=g))
    rng = np.random.default_rng(rank)
    eps = [(int(i), int(e), int(rng.integers(1, T_MAX + 1))) for i in range(N_ENV) for e in range(E_SLOTS)
           if rng.random() < 0.5 + 0.3 * rank]
    return rec, eps


def _expected(rank):
    rec, eps = _fake_records(rank)
    out = []
    for i, e, L in eps:
        out.append(dict(env_id=i, obs=rec["obs"][i, e, :L + 1].numpy(), action=rec["action"][i, e, :L].numpy(),
                        reward=rec["reward"][i, e, :L].numpy(), child=rec["child"][i, e, :L].numpy(),
                        value=rec["value"][i, e, :L].numpy()))
    return out


def _check_episodes(got, want, rank):
    assert len(got) == len(want)
    for g, w in zip(got, want):
        assert g["rank"] == rank and g["env_id"] == w["env_id"]
        assert np.array_equal(g["obs_segment"], w["obs"])
        assert np.array_equal(g["action_segment"], w["action"].astype(np.int64))
        assert np.array_equal(g["reward_segment"], w["reward"])
        assert np.array_equal(g["visits"], w["child"].astype(np.int64))
        tot = w["child"].sum(axis=1, keepdims=True).astype(np.float64)
        tot[tot == 0] = 1e-6
        assert np.array_equal(g["child_visit_segment"], w["child"] / tot)  # store_search_stats, float64
        assert np.array_equal(g["root_value_segment"], w["value"])
        assert g["to_play_segment"].shape == (len(w["action"]),)


def _traj_worker(rank, world, port, out_dir):
    from lightzero_amd.trajectory import all_gather_packed, allreduce_stats, pack_episodes
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rec, eps = _fake_records(rank)
        packed, index = pack_episodes(rec["obs"], rec["action"], rec["reward"], rec["child"], rec["value"], eps)
        blocks = all_gather_packed(packed, index)
        stats = allreduce_stats(10.0 * (rank + 1), float(len(eps)), 0.25, torch.device("cpu"))
        np.savez(os.path.join(out_dir, f"r{rank}.npz"), stats=np.array(stats),
                 **{f"p{r}": p for r, (p, _) in enumerate(blocks)}, **{f"i{r}": i for r, (_, i) in enumerate(blocks)})
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_trajectory_all_gather_gloo_world2(tmp_path):
    from lightzero_amd.trajectory import unpack_episodes
    world = 2
    mp.spawn(_traj_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for me in range(world):
        r = np.load(tmp_path / f"r{me}.npz")
        for rank in range(world):  # every rank holds every rank's episodes
            got = unpack_episodes(r[f"p{rank}"], r[f"i{rank}"], OBS, ACT, rank)
            _check_episodes(got, _expected(rank), rank)
        n_eps = sum(len(_fake_records(k)[1]) for k in range(world))
        assert tuple(r["stats"]) == (30.0, float(n_eps), 0.5)


def test_pack_unpack_round_trip_and_empty():
    from lightzero_amd.trajectory import pack_episodes, unpack_episodes
    rec, eps = _fake_records(0)
    packed, index = pack_episodes(rec["obs"], rec["action"], rec["reward"], rec["child"], rec["value"], eps)
    assert packed.shape == (sum(L + 1 for _, _, L in eps), OBS + 3 + ACT)
    _check_episodes(unpack_episodes(packed.numpy(), index.numpy(), OBS, ACT), _expected(0), 0)
    p0, i0 = pack_episodes(rec["obs"], rec["action"], rec["reward"], rec["child"], rec["value"], [])
    assert p0.shape == (0, OBS + 3 + ACT) and i0.shape == (0, 3)
    assert unpack_episodes(p0.numpy(), i0.numpy(), OBS, ACT) == []
