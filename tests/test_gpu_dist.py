"""Env-sharded collect with the product code on the GPU: two ranks, each a process
running the device collector (search + CartPole + recording, one HIP graph per step) on cuda:0 and
returning its finished episodes through lightzero_amd.trajectory's all-gather and the statistics
sum-reduce over a gloo group (RCCL needs one GPU per rank; the test box has one). Checks that every
rank returns all ranks' episodes, tagged by rank, and the summed statistics."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_world2(tmp_path, env, mode):
    world, port = 2, _free_port()
    procs = []
    for rank in range(world):
        penv = dict(os.environ, RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                    MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.join(REPO, "tests", "dist_gpu_worker.py"),
                                       str(tmp_path), env, mode], env=penv, cwd=REPO))
    codes = [p.wait(timeout=200) for p in procs]
    assert codes == [0] * world, f"worker exit codes {codes}"
    return [np.load(tmp_path / f"out_{r}.npz") for r in range(world)]


@pytest.mark.gpu
@pytest.mark.timeout(240)
def test_sharded_device_collect_gather_to_learner_world2(tmp_path):
    """gather-to-learner (config 5's Breakout shard): rank 0 receives both ranks' episodes, rank 1 none;
    the summed statistics count exactly the episodes the learner received"""
    outs = _run_world2(tmp_path, "breakout", "gather")
    r0, r1 = outs
    assert set(r0["ranks"].tolist()) == {0, 1} and np.all(np.diff(r0["ranks"]) >= 0)
    assert np.array_equal(r0["lens"][r0["ranks"] == 0], r0["own"])
    assert int(r1["sent"]) > 0 and tuple(r0["shape"]) == (1, 64, 64)
    for o in outs:
        assert int(o["world"]) == 2 and int(o["total_episodes"]) == len(r0["ranks"])
        assert int(o["total_envstep"]) == int(r0["envstep"]) + int(r1["envstep"])


@pytest.mark.gpu
@pytest.mark.timeout(240)
@pytest.mark.parametrize("env", ["cartpole", "breakout"])
def test_sharded_device_collect_all_gather_world2(tmp_path, env):
    """env: config 2's CartPole shard, or config 5's Breakout shard (conv search, u8 image frames)"""
    world = 2
    outs = _run_world2(tmp_path, env, "all_gather")
    # every rank holds the same gathered set: both ranks' episodes, in rank order
    assert np.array_equal(outs[0]["ranks"], outs[1]["ranks"]) and np.array_equal(outs[0]["lens"], outs[1]["lens"])
    assert set(outs[0]["ranks"].tolist()) == set(range(world))
    assert np.all(np.diff(outs[0]["ranks"]) >= 0)
    for r in range(world):
        mine = outs[0]["lens"][outs[0]["ranks"] == r]
        assert np.array_equal(mine, outs[r]["own"]), f"rank {r}'s episodes differ after the all-gather"
    assert np.array_equal(outs[0]["sums"], outs[1]["sums"])
    assert tuple(outs[0]["shape"]) == ((1, 64, 64) if env == "breakout" else (4,))
    tot = sum(int(o["envstep"]) for o in outs)
    for o in outs:
        assert int(o["world"]) == world
        assert int(o["total_envstep"]) == tot
        assert int(o["total_episodes"]) == len(outs[0]["ranks"])
