"""Worker of tests/test_gpu_dist.py: one rank of an env-sharded device collect on cuda:0 (the one
GPU of the test box; every rank shares it), trajectories all-gathered over a gloo group. Reads
RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT from the environment, writes out_<rank>.npz."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from lightzero_amd.collector import DeviceCollector  # noqa: E402


def main():
    out_dir = sys.argv[1]
    env = sys.argv[2] if len(sys.argv) > 2 else "cartpole"
    dst = 0 if len(sys.argv) > 3 and sys.argv[3] == "gather" else None  # gather-to-learner: rank 0 receives
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda", 0)
        if env == "cartpole":
            model = bench.build_model(dev, False, seed=0)
            col = DeviceCollector(model, 16, 8, device=dev, seed=bench.shard_seed(rank), graph=True, poll_every=4,
                                  episode_slots=16)
        else:  # config 5's shard: conv MuZeroModel + the Breakout stand-in env, u8 frames on the wire
            model = bench.build_conv_model(dev, seed=0)
            col = DeviceCollector(model, 16, 8, device=dev, seed=bench.shard_seed(rank), graph=True, poll_every=4,
                                  episode_slots=8, max_episode_steps=150, env="breakout")
        col.collect(n_episode=4, dst=dst)  # warm-up collect (returned over the group too)
        eps_all, st_all = col.collect(n_episode=4, group=None, dst=dst)
        if dst is not None and rank != dst:
            assert eps_all == [] and st_all["collective"]["bytes_received"] == 0
            np.savez(os.path.join(out_dir, f"out_{rank}.npz"), sent=st_all["collective"]["bytes_sent"],
                     envstep=st_all["envstep"], total_envstep=st_all["total_envstep"],
                     total_episodes=st_all["total_episodes"], world=st_all["world"])
            return
        ranks = np.array([e["rank"] for e in eps_all], np.int64)
        lens = np.array([len(e["action_segment"]) for e in eps_all], np.int64)
        own = np.array([len(e["action_segment"]) for e in eps_all if e["rank"] == rank], np.int64)
        # a checksum of every episode's first observation frame and of its actions (equal on every rank)
        sums = np.array([float(e["obs_segment"].astype(np.float64).sum()) + float(e["action_segment"].sum())
                         for e in eps_all], np.float64)
        shape = np.array(eps_all[0]["obs_segment"].shape[1:], np.int64)
        np.savez(os.path.join(out_dir, f"out_{rank}.npz"), ranks=ranks, lens=lens, own=own, sums=sums, shape=shape,
                 envstep=st_all["envstep"], total_envstep=st_all["total_envstep"],
                 total_episodes=st_all["total_episodes"], world=st_all["world"])
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
