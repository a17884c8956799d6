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
