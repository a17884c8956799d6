"""Probe: can two ranks of an RCCL ("nccl") process group share the one GPU of the test box? Spawns 2 ranks on
cuda:0, runs one all_gather and one batch_isend_irecv; prints what RCCL says."""
import os
import subprocess
import sys

import torch
import torch.distributed as dist


def worker():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    x = torch.full((4,), float(rank), device=dev)
    out = [torch.empty_like(x) for _ in range(world)]
    dist.all_gather(out, x)
    print(f"rank {rank} all_gather", [float(o[0]) for o in out], flush=True)
    buf = torch.empty(8, dtype=torch.uint8, device=dev)
    if rank == 1:
        ops = [dist.P2POp(dist.isend, torch.arange(8, dtype=torch.uint8, device=dev), 0)]
    else:
        ops = [dist.P2POp(dist.irecv, buf, 1)]
    for r in dist.batch_isend_irecv(ops):
        r.wait()
    torch.cuda.synchronize()
    if rank == 0:
        print("rank 0 received", buf.tolist(), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    if os.environ.get("RANK") is not None:
        worker()
        sys.exit(0)
    procs = [subprocess.Popen([sys.executable, __file__], env=dict(os.environ, RANK=str(r), LOCAL_RANK=str(r),
                                                                     WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                                                                     MASTER_PORT="29533"))
             for r in range(2)]
    codes = [p.wait(timeout=120) for p in procs]
    print("exit codes", codes)
