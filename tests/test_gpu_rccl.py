"""GPU: the trajectory return through RCCL (backend "nccl" on ROCm), not gloo's host copies.

The box has one GPU and RCCL takes one GPU per rank, so this is a world-size-1 RCCL group bound to
cuda:0 (`device_id`, eager communicator init): the same calls the 8-GPU node makes — the device u8 / f32 /
i64 trajectory payload in one flat byte buffer through all_gather and through gather-to-learner
(point-to-point), the float64 statistics all-reduce and bench's max-reduce of the elapsed time — on
device tensors, before the driver's first SCALE run (reference
lzero/worker/muzero_collector.py:709-712). The multi-rank exchange itself is covered with gloo (tests/
test_dist.py, tests/test_gpu_dist.py).
"""
import numpy as np
import pytest
import torch
import torch.distributed as dist

import bench

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


@pytest.fixture(scope="module")
def rccl_group():
    assert not dist.is_initialized()
    dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1, device_id=DEV)
    try:
        assert dist.get_backend() == "nccl"
        yield
    finally:
        dist.destroy_process_group()


def _collector(n=16, S=8, seed=3):
    from lightzero_amd.collector import DeviceCollector
    model = bench.build_conv_model(DEV, seed=0)
    return DeviceCollector(model, n, S, device=DEV, seed=seed, graph=True, poll_every=4, episode_slots=8,
                           max_episode_steps=150, env="breakout")


@pytest.mark.timeout(240)
@pytest.mark.parametrize("dst", [None, 0])
def test_breakout_collect_blocks_over_rccl(rccl_group, dst):
    """DeviceCollector(env="breakout").collect_blocks under the RCCL group: the returned device blocks
    (u8 frames, f32 scalars, i64 index) equal the locally packed ones bit for bit, the statistics are
    all-reduced on the device, and the stats name the backend and the collective's time"""
    from lightzero_amd.trajectory import pack_episodes
    col = _collector()
    for _ in range(80):  # (stand-in Breakout episodes last tens of steps)
        col.step()
    counts = col.ep_count.cpu().numpy().astype(np.int64)
    ln = col.ep_len.cpu().numpy()
    todo = [(i, k % col.E, int(ln[i, k % col.E])) for i in range(col.n) for k in range(int(col._consumed[i]),
                                                                                    int(counts[i]))]
    assert todo, "no finished episodes after 80 steps"
    ref = pack_episodes(col.rec_frames, col.rec_action, col.rec_reward, col.rec_visits, col.rec_value, todo,
                        col.rec_pred, col.env.frame_scale, ep_return=col.ep_return)
    blocks, st = col.gather_blocks(to_host=False, dst=dst)
    (b,) = blocks
    assert b.frames.is_cuda and b.frames.dtype == torch.uint8 and b.scalars.dtype == torch.float32
    assert b.index.dtype == torch.int64
    assert torch.equal(b.frames, ref.frames) and torch.equal(b.scalars, ref.scalars)
    assert torch.equal(b.index.cpu(), ref.index)
    c = st["collective"]
    assert c["backend"] == "nccl" and c["ms"] > 0 and c["bytes_sent"] > 0
    assert c["mode"] == ("all_gather" if dst is None else "gather(dst=0)")
    assert st["world"] == 1 and st["total_episodes"] == len(todo) and st["total_envstep"] == 80 * col.n


def test_rccl_all_gather_packed_and_gather_packed_device_dtypes(rccl_group):
    """the flat wire buffer through RCCL for every payload dtype the collectors record (CartPole's f32
    vectors, Atari's u8 frames), empty blocks included"""
    from lightzero_amd.trajectory import TrajBlock, all_gather_packed, gather_packed
    g = torch.Generator(device=DEV).manual_seed(5)
    for fshape, fdtype in (((4,), torch.float32), ((1, 64, 64), torch.uint8)):
        for rows, n_ep in ((37, 3), (0, 0)):
            if fdtype == torch.uint8:
                frames = torch.randint(0, 256, (rows,) + fshape, generator=g, device=DEV, dtype=torch.uint8)
            else:
                frames = torch.randn((rows,) + fshape, generator=g, device=DEV)
            sc = torch.randn((rows, 7), generator=g, device=DEV)
            ix = torch.randint(0, 1 << 40, (n_ep, 3), generator=g, device=DEV, dtype=torch.int64)
            blk = TrajBlock(frames, sc, ix, 0.5)
            for fn in (all_gather_packed, lambda b, to_host: gather_packed(b, 0, to_host=to_host)):
                (got,) = fn(blk, to_host=False)
                assert got.frames.dtype == fdtype and got.frames.shape == frames.shape
                assert torch.equal(got.frames.to(DEV), frames) and torch.equal(got.scalars.to(DEV), sc)
                assert torch.equal(got.index.to(DEV), ix) and got.frame_scale == 0.5


def test_rccl_statistics_and_max_reduce(rccl_group):
    from lightzero_amd.trajectory import allreduce_stats
    assert allreduce_stats(123.0, 4.0, 0.25, DEV) == (123.0, 4.0, 0.25)
    t = torch.tensor([1.25], dtype=torch.float64, device=DEV)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    assert float(t.item()) == 1.25
    assert bench.slowest_rank_seconds(1.5, 1, DEV) == 1.5
