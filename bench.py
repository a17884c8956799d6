"""bench.py — MCTS simulations/sec of the batched MuZero search (BASELINE.json metric).

Workload (BASELINE.json configs[1]): CartPole-v0 MuZero, 256 envs x 50 simulations per GPU,
MuZeroModelMLP (latent 128, support 601, residual dynamics, BN) with random weights, synthetic
observations. One step = one self-play search pass over the batch exactly as
MuZeroPolicy._forward_collect runs it (lzero/policy/muzero.py:617-690): initial_inference ->
Roots.prepare (Dirichlet-mixed priors) -> MuZeroMCTSCtree.search (50 simulations) -> root
visit distributions and values. Inputs are resident in HBM before the timed region.

Multi-GPU: one process per GPU. Under torchrun the ranks come from the environment;
`python bench.py --gpus N` started directly launches the N rank processes itself (launch_ranks:
fresh interpreters, the parent never touches the GPU). Every rank searches its own 256 envs (envs
are independent trees: weak scaling, no collective in the data path). value = all ranks' sims /
the slowest rank's time. `--step collect` runs the device collector per rank and ends the timed
region with the trajectory return (device pack + the flat byte buffer gathered to the learner rank
over RCCL, or all-gathered with --traj all_gather + statistics sum, trajectory.py); with one GPU the
collectives still run, in a one-rank RCCL group (--rccl-world1).
`--dry-run` checks the launch on gloo without a GPU.

Extra objects on the JSON line:
  roofline     - dominant HIP kernel of the step: algorithmic work per launch / its live HIP-event
                 duration vs the peak (fused: fp32 FLOPs vs the fp32 VALU peak — the network runs on
                 v_pk_fma_f32, MFMA utilisation 0 —, plus the L2 weight stream; generic: bytes vs
                 HBM); traffic = PMC HBM bytes per launch from the committed profile
                 (profiles/pmc_latest.json); profiles/ holds the matching rocprof stats
  cpu_baseline - the oracle's bit-exact CPU restatement of the reference ctree ("port"; the
                 reference never ships to the GPU box) in BASELINE.md's four variants (tree only on
                 1 thread / the CPU share; the reference search architecture with the network on the
                 GPU / on the CPU share), the host's nproc and CPU model, and the reference-vs-port
                 calibration ratios measured in the build container (profiles/cpu_calibration.json).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP32_PEAK_TFLOPS = 157.3  # MI355X fp32 VALU peak (= the f32 MFMA rate on gfx950, MI355X_MICROARCH.md)
L2_PEAK_TBS = 34.5  # aggregate L2 bandwidth, 8 XCDs (MI355X_MICROARCH.md)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--envs", type=int, default=256)
    p.add_argument("--sims", type=int, default=50)
    p.add_argument("--rng", choices=["glibc", "philox"], default="glibc")
    p.add_argument("--path", choices=["fused", "generic"], default="fused",
                   help="fused: one lzm_search_mlp launch per search; generic: HIP tree kernels around the "
                        "PyTorch network (any model)")
    p.add_argument("--graph", type=int, default=1, help="generic path: replay each search as one HIP graph")
    p.add_argument("--step", choices=["graph", "python", "collect"], default="graph",
                   help="graph: the collect-time search pass as one HIP graph (lightzero_amd.collect."
                        "DeviceSearchStep); python: the same sequence driven call by call from Python; "
                        "collect: one full env step of the device collector (search + action selection + "
                        "CartPole step + recording, lightzero_amd.collector.DeviceCollector)")
    p.add_argument("--cpu-baseline-secs", type=float, default=30.0,
                   help="total CPU-baseline sample over the four variants")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--zero-heads", action="store_true", help="reference zero-init last layers (all-tie search)")
    p.add_argument("--workload", choices=["cartpole", "breakout"], default="cartpole",
                   help="cartpole: BASELINE.json config 2 (the headline); breakout: config 5's per-GPU shard "
                        "(conv MuZeroModel, 4x64x64 frames, 4 actions; 2048 envs = 256 per GPU x 8)")
    p.add_argument("--secondary", choices=["breakout", "none"], default="breakout",
                   help="after the headline, also time config 5's sharded collect step (Breakout stand-in env, "
                        "search + env + recording + trajectory all-gather) and report it in the line's 'config5'")
    p.add_argument("--traj", choices=["gather", "all_gather"], default="gather",
                   help="collect steps' trajectory return: gather = to the learner rank 0 alone (each rank sends its "
                        "flat byte buffer once, point to point); all_gather = to every rank")
    p.add_argument("--rccl-world1", type=int, default=1,
                   help="N = 1: still run under a one-rank RCCL process group, so the collect steps' trajectory "
                        "return and statistics all-reduce go through RCCL as on the 8-GPU node (0: no group)")
    p.add_argument("--configs", default="1,3,4",
                   help="with one GPU, also time these BASELINE.json configs into the line ('config1', 'config3', "
                        "'config4' objects, each with its roofline and CPU baseline); 'none' skips them")
    p.add_argument("--dry-run", action="store_true",
                   help="launcher check without a GPU: the ranks join a gloo group and rank 0 prints who joined")
    return p.parse_args()


def launch_ranks(n, argv):
    """`bench.py --gpus N` run directly (not under torchrun): start N fresh rank processes with
    RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set (one per GPU, rendezvous on 127.0.0.1) and wait
    for them; rank 0 prints the line. This parent never initialises the GPU (nothing before this
    point calls into HIP) and starts children instead of re-exec'ing. A failing rank stops the
    others; returns the first failing exit code (0 when every rank succeeded)."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    try:
        pending = set(range(n))
        while pending:
            for r in sorted(pending):
                c = procs[r].poll()
                if c is None:
                    continue
                pending.discard(r)
                if c != 0 and rc == 0:
                    rc = c if c > 0 else 128 - c
                    for q in pending:
                        procs[q].terminate()
            time.sleep(0.05)
    finally:
        for pr in procs:
            if pr.poll() is None:
                pr.kill()
                pr.wait()
    return rc


def rank_info(rank, local, device):
    d = {"rank": rank, "local_rank": local}
    if device is not None:
        props = torch.cuda.get_device_properties(device)
        d.update(device=str(device), name=props.name, pci_bus_id=getattr(props, "pci_bus_id", None))
    return d


def dry_run(world, rank, local):
    """The launch logic without a GPU: every rank joins a gloo group (as the real ranks join
    RCCL), the ranks are gathered and rank 0 prints them on one JSON line."""
    if world > 1:
        dist.init_process_group("gloo")
        ranks = [None] * world
        dist.all_gather_object(ranks, rank_info(rank, local, None))
    else:
        ranks = [rank_info(rank, local, None)]
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "ranks": ranks}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def _random_bn(m, seed):
    """random BatchNorm statistics so eval-mode BN is not the identity"""
    g = torch.Generator().manual_seed(seed)
    for mod in m.modules():
        if isinstance(mod, (torch.nn.BatchNorm1d, torch.nn.BatchNorm2d)):
            with torch.no_grad():
                mod.running_mean.copy_(torch.randn(mod.running_mean.shape, generator=g) * 0.1)
                mod.running_var.copy_(torch.rand(mod.running_var.shape, generator=g) * 0.5 + 0.75)
                mod.weight.copy_(torch.rand(mod.weight.shape, generator=g) * 0.5 + 0.75)
                mod.bias.copy_(torch.randn(mod.bias.shape, generator=g) * 0.1)


def build_model(device, zero_heads, seed):
    from lightzero_amd.model_mlp import cartpole_muzero_model
    torch.manual_seed(seed)
    m = cartpole_muzero_model(random_heads=not zero_heads)
    _random_bn(m, seed + 1)
    return m.to(device).eval()


def build_conv_model(device, seed=0, zero_heads=False):
    """config 5's network: the restated conv MuZeroModel at Breakout's shapes (atari_muzero_config.py:
    obs 4x64x64, 4 actions, support 601), random weights (non-zero heads unless zero_heads) and BN stats"""
    from lightzero_amd.model_conv import atari_muzero_model
    torch.manual_seed(seed)
    m = atari_muzero_model(last_linear_layer_init_zero=bool(zero_heads))
    _random_bn(m, seed + 1)
    return m.to(device).eval()


def build_ez_model(device, seed=0, zero_heads=False):
    """config 3's network: the restated conv EfficientZeroModel at Pong's shapes (atari_efficientzero_config.py:
    obs 4x64x64, 6 actions, LSTM 512, support 101), random weights (non-zero heads unless zero_heads) and BN
    stats"""
    from lightzero_amd.model_conv import atari_efficientzero_model
    torch.manual_seed(seed)
    m = atari_efficientzero_model(last_linear_layer_init_zero=bool(zero_heads))
    _random_bn(m, seed + 1)
    return m.to(device).eval()


WORKLOADS = {
    # name: (actions, observation shape, device env of the collect step, support_scale)
    "cartpole": (2, (4,), "cartpole", 300),
    "breakout": (4, (4, 64, 64), "breakout", 300),
    "pong": (6, (4, 64, 64), "pong", 50),
}


def synthetic_obs(workload, B, rng):
    """config 2: N(0,1) [B, 4]; config 5: frames U{0..255}/255 [B, 4, 64, 64]"""
    if workload == "cartpole":
        return rng.normal(size=(B, 4)).astype(np.float32)
    return (rng.integers(0, 256, size=(B, 4, 64, 64)).astype(np.float32) / 255.0).astype(np.float32)  # (Atari)


class GraphStep:
    """One collect-time search pass (muzero.py:617-690; efficientzero.py:538-656) as one HIP graph
    (DeviceSearchStep): initial_inference -> Roots.prepare (noise) -> one-launch search -> distributions /
    values; the traverse seeds advance on the device every replay. workload: config 2 / 1 (MLP), config 5
    (conv MuZero: BN-folded initial inference + lzm_search_conv) or config 3 ("pong": conv EfficientZero,
    + lzm_search_conv_ez with the reward LSTM)."""

    def __init__(self, B, S, model, device, rng_mode, seed, workload="cartpole"):
        from lightzero_amd.collect import DeviceSearchStep
        rng = np.random.default_rng(seed)
        A, shape, _, scale = WORKLOADS[workload]
        self.B, self.S = B, S
        self.step = DeviceSearchStep(model, B, S, [list(range(A))] * B, shape, device, noise_weight=0.25, seed=seed,
                                     rng_mode=rng_mode, graph=True, support_scale=scale)
        self.step.set_inputs(obs=torch.from_numpy(synthetic_obs(workload, B, rng)).to(device),
                             noises=torch.from_numpy(rng.dirichlet([0.3] * A, size=B).astype(np.float32)).to(device))
        self.mcts = self.step.mcts
        self.last = None

    def __call__(self):
        out = self.step.step()
        self.last = (out["distributions"], out["values"], None)

    def tree(self):
        return self.step.roots.tree


class CollectStep:
    """One env step of the device collector for every env: search + select_action + CartPole step +
    GameSegment recording, one HIP graph (muzero_collector.py:399-705 per step)."""

    def __init__(self, B, S, model, device, rng_mode, seed, workload="cartpole", dst=0):
        from lightzero_amd.collector import DeviceCollector
        self.B, self.S = B, S
        self.dst = dst  # trajectory return: gather to rank dst (None: all-gather)
        env = WORKLOADS[workload][2]
        # CartPole episodes are short (tens of steps): many slots per env; Breakout stand-in episodes
        # last >= ~17 steps, 400-step limit; Pong stand-in episodes (21 points, hundreds of steps) truncated
        # at 100 steps, so that episodes finish inside a 100-step timed region
        slots, T = {"cartpole": (64, 200), "pong": (8, 100)}.get(env, (8, 400))
        self.col = DeviceCollector(model, B, S, device=device, seed=seed, rng_mode=rng_mode, graph=True,
                                   episode_slots=slots, max_episode_steps=T, env=env)
        self.step = self.col.search
        self.mcts = self.step.mcts
        self.last = None

    def __call__(self):
        self.col.step()
        out = self.col.search.out
        self.last = (out["distributions"], out["values"], None)

    def finish(self, world):
        """the episodes finished since the last call: packed on the device (lzm_episodes_*) and, under a
        process group, returned over it (RCCL over xGMI: gathered to the learner rank, or all-gathered)
        with the step / episode / duration sums (trajectory.py) — the TrajBlocks a learner consumes, no
        host unpacking"""
        blocks, st = self.col.gather_blocks(to_host=False, dst=self.dst)
        c = st["collective"]
        return {"episodes_received": st["episodes"], "episodes_all_ranks": int(st["total_episodes"]),
                "rows_received": st["rows"], "payload_bytes_received": st["payload_bytes"],
                "frame_dtype": str(self.col.rec_frames.dtype).replace("torch.", ""),
                "total_envstep": st["total_envstep"], "world": world,
                "backend": c["backend"] if c else None, "mode": c["mode"] if c else None,
                "collective_ms": round(c["ms"], 3) if c else None,
                "wire_bytes_sent": c["bytes_sent"] if c else None,
                "wire_bytes_received": c["bytes_received"] if c else None}

    def tree(self):
        return self.col.search.roots.tree


class GpuStep:
    """One collect-time search pass (muzero.py:660-690) on the GPU drop-in, driven from Python."""

    def __init__(self, B, S, model, device, rng_mode, graph, seed, fused=True):
        from lightzero_amd.mcts_ctree import MuZeroMCTSCtree
        from lightzero_amd.utils import EasyDict
        from lightzero_amd.tree import SequentialSeeds, set_seed_source
        self.B, self.S, self.model, self.device = B, S, model, device
        MuZeroMCTSCtree.rng_mode = rng_mode
        self.cls = MuZeroMCTSCtree
        cfg = EasyDict(dict(num_simulations=S, discount_factor=0.997, device=device, use_hip_graph=bool(graph),
                            fused_search=bool(fused),
                            model=dict(support_scale=300, categorical_distribution=True)))
        self.mcts = MuZeroMCTSCtree(cfg)
        rng = np.random.default_rng(seed)
        self.obs = torch.from_numpy(rng.normal(size=(B, 4)).astype(np.float32)).to(device)
        self.noises = torch.from_numpy(rng.dirichlet([0.3, 0.3], size=B).astype(np.float32)).to(device)
        self.legal = [[0, 1] for _ in range(B)]
        self.to_play = torch.full((B,), -1, dtype=torch.int32, device=device)
        self.zero = torch.zeros(B, dtype=torch.float32, device=device)
        set_seed_source(SequentialSeeds(seed))
        self.last = None

    def __call__(self):
        with torch.no_grad():
            out = self.model.initial_inference(self.obs)
            roots = self.cls.roots(self.B, self.legal)
            roots.prepare_device(0.25, self.noises, self.zero, out.policy_logits, self.to_play)
            self.mcts.search(roots, self.model, out.latent_state, self.to_play)
            t = roots.tree
            self.last = (t.distributions(), t.values(), t.search_len)
            self._tree = t
            roots.clear()

    def tree(self):
        return self._tree


def kernel_timing(step, n_search=3):
    """Live per-launch durations (HIP events on the launch stream — torch's current stream, the
    one every lzm_* call is enqueued on) of the search kernels over `n_search` searches, plus
    the mean search depth d-bar from the kernels' own search_len output."""
    from lightzero_amd import mcts_ctree as mc
    mcts = step.mcts
    names = ("traverse", "decode_backprop", "search_mlp", "search_conv", "search_conv_ez")
    orig = {n: getattr(mc.DeviceTree, n) for n in names}
    acc = {n: [] for n in names}
    depth = []

    def timed(name, fn):
        def w(self, *a, **k):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            if hasattr(torch.cuda, "_sleep"):
                # keep the stream busy while the host enqueues e0, the launch and e1, so the events
                # bracket the kernel alone (not the host-side launch latency)
                torch.cuda._sleep(200000)
            e0.record()
            fn(self, *a, **k)
            e1.record()
            acc[name].append((e0, e1))
            if name == "traverse":
                depth.append(self.search_len.clone())
        return w

    use_graph = mcts._cfg.get("use_hip_graph", False)
    mcts._cfg.use_hip_graph = False
    for n in names:
        setattr(mc.DeviceTree, n, timed(n, orig[n]))
    # a graph replay runs no Python: time the captured body eagerly (same kernels, same inputs)
    run = step.step._body if isinstance(step, (GraphStep, CollectStep)) else step
    try:
        # d-bar from one recorded search (recording adds per-simulation stores to the fused kernel,
        # so the timed searches below run without it, as the bench step does)
        mcts.record = True
        run()
        if mcts.last_record is not None and not acc["traverse"]:
            depth.append(mcts.last_record.search_len.clone())
        mcts.record = False
        for v in acc.values():
            v.clear()
        for _ in range(n_search):
            run()
        torch.cuda.synchronize()
    finally:
        for n in names:
            setattr(mc.DeviceTree, n, orig[n])
        mcts._cfg.use_hip_graph = use_graph
        mcts.record = False
    ms = {k: float(np.mean([a.elapsed_time(b) for a, b in v])) for k, v in acc.items() if v}
    dbar = float(torch.cat([d.reshape(-1) for d in depth]).float().mean().item())
    return ms, dbar


def mlp_flops_per_sim(H, A, F, V, res=True):
    """2 x multiply-adds of one recurrent_inference row (149,376 MAC at
    H=128, A=2, F=32, V=601)."""
    mac = (H + A) * H + H * H          # fc_dynamics(_1)
    mac += 2 * H * H if res else 0     # fc_dynamics_2
    mac += H * F + F * V               # fc_reward_head
    mac += 2 * H * H                   # fc_prediction_common
    mac += H * F + F * V               # fc_value_head
    mac += H * F + F * A               # fc_policy_head
    return 2 * mac


def conv_flops_per_sim(model, B, device):
    """(all, matrix-pipe) FLOPs of one recurrent_inference row of the conv MuZeroModel / EfficientZeroModel
    (torch FlopCounterMode at batch B: the convolutions are the trunk on the split-fp16 MFMA path, the
    Linears the head MLPs on the VALU). EfficientZero's reward LSTM, which the counter does not see inside
    nn.LSTM, is counted by hand as its gate GEMM, 2 x 4H x (K + H) per row (K = reward planes, H = 512),
    on the matrix pipe too (lzm_ez_lstm_step)."""
    from torch.utils.flop_counter import FlopCounterMode
    lat = torch.zeros(B, 64, 8, 8, device=device)
    act = torch.zeros(B, dtype=torch.int64, device=device)
    ez = hasattr(model.dynamics_network, "lstm")
    with torch.no_grad(), FlopCounterMode(display=False) as fc:
        if ez:
            z = torch.zeros(1, B, model.lstm_hidden_size, device=device)
            model.recurrent_inference(lat, (z, z), act)
        else:
            model.recurrent_inference(lat, act)
    per_op = {str(k): v for k, v in fc.get_flop_counts().get("Global", {}).items()}
    total = fc.get_total_flops() / B
    matrix = sum(v for k, v in per_op.items() if "convolution" in k) / B
    if ez:
        lstm = model.dynamics_network.lstm
        gate = 2.0 * 4 * lstm.hidden_size * (lstm.input_size + lstm.hidden_size)
        total += gate - sum(v for k, v in per_op.items() if "lstm" in k) / B
        matrix += gate
    return total, matrix


def shard_seed(rank):
    """Each rank searches its own envs: per-rank synthetic inputs and traverse seeds."""
    return 1000 + rank


def slowest_rank_seconds(elapsed, world, device):
    """The job's time is the slowest rank's (max-reduce over the process group when one is initialised;
    envs are independent trees, nothing crosses ranks in the search's data path)."""
    if world == 1 and not (dist.is_available() and dist.is_initialized()):
        return elapsed
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def whole_job_rate(B, S, steps, world, seconds):
    """Simulations of all ranks (B envs x S sims per rank per step) per second."""
    return world * B * S * steps / seconds


def roots_per_workgroup(B, device):
    """The library's choice (lzm_kernels.hip roots_per_wg): smallest of 1, 2, 4, 8 that fits one
    workgroup per CU; LZM_ROOTS_PER_WG overrides."""
    env = os.environ.get("LZM_ROOTS_PER_WG")
    if env in ("1", "2", "4", "8"):
        return int(env)
    cus = torch.cuda.get_device_properties(device).multi_processor_count
    return next((r for r in (1, 2, 4) if -(-B // r) <= cus), 8)


def _lib_kernel_floats(H=128, A=2, F=32, V=601, res=1):
    """floats of the weight-streaming kernel's layout (lzm_mlp_kernel_floats, minus the resident
    kernel's blocks that follow it for the config-2 shape: lzm_search_res.h res_block_floats)"""
    from lightzero_amd import _lib
    n = int(_lib.load().lzm_mlp_kernel_floats(H, A, F, V, res))
    if (H, F, V, res) == (128, 32, 601, 1) and A <= 32:
        n -= 6 * 16384 + 4096 + 8192 + 2 * 20480 + 1024 + 6 * 128 + 32 + 64 + 2 * 604 + 32 + A * 128
    return n


def pmc_traffic(kernel):
    """HBM bytes per launch from the COMMITTED PMC passes (profiles/pmc_latest.json, built by
    tools/pmc_latest.py from tools/profile_round.sh on the GPU box), not measured in this run: 2 x FETCH_SIZE +
    WRITE_SIZE of that kernel, or None."""
    path = os.path.join(REPO, "profiles", "pmc_latest.json")
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return None
    base = kernel.split("<")[0]
    for e in (d.get("kernels") or {}).values():
        if e.get("kernel", "").split("(")[0].split("<")[0].endswith(base) and e.get("traffic_bytes"):
            return e["traffic_bytes"]
    return None


def pmc_source():
    """where roofline.traffic comes from: the committed PMC file, its pass directory, build date and head"""
    try:
        d = json.load(open(os.path.join(REPO, "profiles", "pmc_latest.json")))
    except (OSError, ValueError):
        return None
    return dict({"file": "profiles/pmc_latest.json", "measured_in_this_run": False}, **(d.get("source") or {}))


def algorithmic_bytes(B, A, H, V, dbar):
    """Bytes each kernel must move per launch (this layout: 16-B node records).
    traverse: per level the parent's stat+meta records (32 B) and A child stat records (16 A),
    path + action writes (8 B); per root the six result words (28 B).
    decode_backprop: two support rows (8 V) + policy logits (4 A) + the new latent row read and
    filed into the pool (8 H) + A child records written (32 A) + leaf meta (16) + the backup
    read-modify-write of (d+1) stat records and their meta (48 (d+1)) + min-max (16)."""
    trav = B * (dbar * (32 + 16 * A + 8) + 28)
    dec = B * (8 * V + 4 * A + 8 * H + 32 * A + 16 + 48 * (dbar + 1) + 16)
    return {"traverse": trav, "decode_backprop": dec}


def survey_hbm(sims_per_s, A, H, V, dbar, extra=0, note=None):
    """BASELINE.md's HBM-roofline fraction: sims/s x SURVEY.md §8(d)'s algorithmic bytes per simulation / 8 TB/s,
    with d-bar the measured mean search_len. Bytes per simulation: select d(16A + 12), leaf record 16, gather
    4H + 4, scatter 4H, decode 8V + 4A, expand 16A + 16, backup 24(d + 1) + 8 (+ extra: EfficientZero's LSTM
    state, 4 x 512 x 4 B). H is the latent's float count: 128 for the MLP configs, 64 x 8 x 8 = 4096 for the conv
    configs (§8(d)'s C3 / C5 figures used 1024, a 64 x 4 x 4 latent: the reference's DownSample ends at 8 x 8 for
    64 x 64 frames, common.py:258-262)."""
    per_sim = dbar * (16 * A + 12) + 16 + (4 * H + 4) + 4 * H + (8 * V + 4 * A) + (16 * A + 16) + 24 * (dbar + 1) + 8 \
        + extra
    gbs = sims_per_s * per_sim / 1e9
    out = {"definition": "sims/s x SURVEY.md 8(d) bytes/sim / peak HBM (BASELINE.md)", "bytes_per_sim": round(per_sim, 1),
           "mean_search_len": round(dbar, 3), "A": A, "H": H, "V": V, "achieved": round(gbs, 2), "peak": HBM_PEAK_GBS,
           "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 6)}
    if note:
        out["note"] = note
    return out


def az_mean_depth(m, B, S):
    """AlphaZero: the mean simulation depth from the exported trees — every simulation adds one visit to each
    non-root node of its path, so sum over non-root nodes of the visits / (B S) is the mean depth"""
    visit, _, _, nn = m.export_tree(B)  # [B][1 + 9 (S + 1)] node visits, root first; nodes in use per board
    used = torch.arange(visit.shape[1], device=visit.device).unsqueeze(0) < nn.unsqueeze(1)
    used[:, 0] = False
    return float((visit.double() * used).sum().item() / (B * S))


def host_cpu_info():
    """The box's host CPU as the CPU-baseline line records it: nproc (os.cpu_count, the whole
    machine), the affinity mask, the job's thread share (OMP_NUM_THREADS, which the GPU pool sets
    per GPU) and the model name."""
    info = {"nproc": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)),
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}
    try:
        with open("/proc/cpuinfo") as f:
            info["model"] = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), None)
    except OSError:
        info["model"] = None
    return info


def share_threads():
    """Threads for the all-cores variants: the job's CPU share (OMP_NUM_THREADS when set — the
    pool gives each GPU job 16 — else the affinity mask)."""
    env = os.environ.get("OMP_NUM_THREADS")
    n = int(env) if env and env.isdigit() and int(env) > 0 else len(os.sched_getaffinity(0))
    return max(1, min(n, len(os.sched_getaffinity(0))))


def cpu_tree_only(B, A, S, threads, secs):
    """BASELINE.md CPU plan (a)/(b): the oracle's bit-exact restatement of the reference ctree
    (oracle/lz_oracle.c, cnode.cpp restated), tree only — prepare + S x (cbatch_traverse,
    cbatch_backpropagate) with scripted network outputs — envs partitioned over `threads`
    pthreads (shard-local tie-break streams). Returns (sims/s, searches, seconds)."""
    from oracle.oracle import lib
    L = lib()
    n = 1
    while True:  # grow the sample until it fills at least half the budget (thread start-up aside)
        el = L.lzo_bench_tree_only(B, A, S, threads, n, 12345)
        if el >= 0.5 * secs or n >= 1 << 24:
            return B * S * n / el, n, el
        n = max(n + 1, int(n * min(64.0, 0.8 * secs / max(el, 1e-6))))


def cpu_reference_search(B, S, model, secs, threads, device=None):
    """BASELINE.md CPU plan (c)/(d): the reference's search architecture (mcts_ctree.py:228-321):
    the host tree (the oracle's restatement of cnode.cpp, single-threaded as the reference's
    ctree) + the network through PyTorch + InverseScalarTransform + the host gather of
    latent[x][y] and the list glue. device=None: the network on torch-CPU with `threads` threads
    (plan (d)); a GPU device: the network on the GPU with per-simulation H2D / D2H copies, as
    LightZero runs it with cuda=True (plan (c)). Returns (sims/s, searches, seconds)."""
    from oracle.oracle import OracleTree
    torch.set_num_threads(threads)
    dev = torch.device("cpu") if device is None else device
    rng = np.random.default_rng(0)
    obs = torch.from_numpy(rng.normal(size=(B, 4)).astype(np.float32)).to(dev)
    support = torch.arange(-300, 301, dtype=torch.float64, device=dev).unsqueeze(0)

    def inv(logits):
        p = torch.softmax(logits, dim=1)
        v = p.mul_(support).sum(1, keepdim=True)
        tmp = (torch.sqrt(1 + 4 * 0.001 * (torch.abs(v) + 1 + 0.001)) - 1) / (2 * 0.001)
        return (torch.sign(v) * (tmp * tmp - 1)).float()

    n, t0 = 0, time.perf_counter()
    with torch.no_grad():
        while True:
            out = model.initial_inference(obs)
            tree = OracleTree(B, 2, S)
            tree.set_delta(np.float32(0.01))
            noises = rng.dirichlet([0.3, 0.3], size=B).astype(np.float32)
            tree.prepare(np.float32(0.25), noises, np.zeros(B, np.float32), out.policy_logits.cpu().numpy(),
                         np.full(B, -1, np.int32))
            pool = [out.latent_state.cpu().numpy()]
            tp = np.full(B, -1, np.int32)
            for k in range(S):
                x, y, a, vtp, _ = tree.traverse(19652, np.float32(1.25), np.float32(0.997), k, tp)
                lat = torch.from_numpy(np.asarray([pool[ix][iy] for ix, iy in zip(x, y)])).to(dev)
                o = model.recurrent_inference(lat, torch.from_numpy(a.astype(np.int64)).to(dev))
                pool.append(o.latent_state.cpu().numpy())
                tree.backprop(k + 1, np.float32(0.997), inv(o.reward).cpu().numpy().reshape(-1),
                              inv(o.value).cpu().numpy().reshape(-1), o.policy_logits.cpu().numpy(), vtp)
            n += 1
            el = time.perf_counter() - t0
            if el >= secs:
                return n * B * S / el, n, el


def cpu_reference_search_conv(kind, B, S, model, secs, threads, device=None, seed=0):
    """The reference's search architecture at the conv Atari configs (mcts_ctree.py:228-321 for
    MuZero / config 5, :696-827 for EfficientZero / config 3): the host tree (the oracle's bit-exact
    restatement of ctree_muzero / ctree_efficientzero, single-threaded as the reference's ctree), the
    host gather of latent[x][y] (and of the LSTM state for EZ, zeroed where search_len % 5 == 0), the
    network through PyTorch and InverseScalarTransform. device=None: the network on torch-CPU with
    `threads` threads; a GPU device: on the GPU with per-simulation H2D / D2H copies (LightZero with
    cuda=True). At least one whole search is timed. Returns (sims/s, searches, seconds)."""
    from oracle.oracle import OracleTree
    torch.set_num_threads(threads)
    dev = torch.device("cpu") if device is None else device
    model = model.to(dev).eval()
    A = model.action_space_size
    ez = kind == "ez"
    scale = 50 if ez else 300
    rng = np.random.default_rng(seed)
    obs = torch.from_numpy(synthetic_obs("breakout", B, rng)).to(dev)
    support = torch.arange(-scale, scale + 1, dtype=torch.float64, device=dev).unsqueeze(0)

    def inv(logits):
        p = torch.softmax(logits, dim=1)
        v = p.mul_(support).sum(1, keepdim=True)
        tmp = (torch.sqrt(1 + 4 * 0.001 * (torch.abs(v) + 1 + 0.001)) - 1) / (2 * 0.001)
        return (torch.sign(v) * (tmp * tmp - 1)).float().cpu().numpy().reshape(-1)

    n, t0 = 0, time.perf_counter()
    with torch.no_grad():
        while True:
            out = model.initial_inference(obs)
            tree = OracleTree(B, A, S, ez=ez)
            tree.set_delta(np.float32(0.01))
            noises = rng.dirichlet([0.3] * A, size=B).astype(np.float32)
            tree.prepare(np.float32(0.25), noises, np.zeros(B, np.float32), out.policy_logits.cpu().numpy(),
                         np.full(B, -1, np.int32))
            pool = [out.latent_state.cpu().numpy()]
            if ez:
                hpool = [out.reward_hidden_state[0].reshape(B, -1).cpu().numpy()]
                cpool = [out.reward_hidden_state[1].reshape(B, -1).cpu().numpy()]
            tp = np.full(B, -1, np.int32)
            for k in range(S):
                x, y, a, vtp, slen = tree.traverse(19652, np.float32(1.25), np.float32(0.997), k, tp)
                lat = torch.from_numpy(np.asarray([pool[ix][iy] for ix, iy in zip(x, y)])).to(dev)
                act = torch.from_numpy(a.astype(np.int64)).to(dev)
                if ez:
                    h = torch.from_numpy(np.asarray([hpool[ix][iy] for ix, iy in zip(x, y)])).to(dev).unsqueeze(0)
                    c = torch.from_numpy(np.asarray([cpool[ix][iy] for ix, iy in zip(x, y)])).to(dev).unsqueeze(0)
                    o = model.recurrent_inference(lat, (h, c), act)
                    reset = (slen % 5 == 0).astype(np.int32)
                    keep = (1 - reset).astype(np.float32)[:, None]
                    hpool.append(o.reward_hidden_state[0].reshape(B, -1).cpu().numpy() * keep)
                    cpool.append(o.reward_hidden_state[1].reshape(B, -1).cpu().numpy() * keep)
                    pool.append(o.latent_state.cpu().numpy())
                    tree.backprop(k + 1, np.float32(0.997), inv(o.value_prefix), inv(o.value),
                                  o.policy_logits.cpu().numpy(), vtp, reset)
                else:
                    o = model.recurrent_inference(lat, act)
                    pool.append(o.latent_state.cpu().numpy())
                    tree.backprop(k + 1, np.float32(0.997), inv(o.reward), inv(o.value), o.policy_logits.cpu().numpy(),
                                  vtp)
            n += 1
            el = time.perf_counter() - t0
            if el >= secs:
                return n * B * S / el, n, el


def cpu_baseline_conv(kind, B, S, model_gpu, secs, device):
    """CPU baseline of a conv config (3: Pong EZ, 5: Breakout MZ per GPU): BASELINE.md's variants of the
    bit-exact port — (a)/(b) the tree alone on 1 thread / the CPU share, (c) the reference search
    architecture with the network on this GPU (one host thread, per-simulation H2D / D2H), (d) the same
    with the network on torch-CPU over the share. `value` is (d). The conv network costs ≈ 25 MFLOP per
    simulation, so (c) and (d) time at least one whole 256 x 50 search each."""
    import copy
    T = share_threads()
    A = model_gpu.action_space_size
    var = {}
    v, n, el = cpu_tree_only(B, A, S, 1, 0.1 * secs)
    var["a_tree_only_1t"] = {"value": round(v, 1), "cores": 1, "searches": n, "seconds": round(el, 2)}
    v, n, el = cpu_tree_only(B, A, S, T, 0.1 * secs)
    var["b_tree_only_share"] = {"value": round(v, 1), "cores": T, "searches": n, "seconds": round(el, 2)}
    v, n, el = cpu_reference_search_conv(kind, B, S, model_gpu, 0.3 * secs, 1, device=device)
    var["c_ref_arch_gpu_net_1t"] = {"value": round(v, 1), "cores": 1, "searches": n, "seconds": round(el, 2),
                                    "network": "this GPU (PyTorch-ROCm), per-simulation H2D/D2H"}
    model_cpu = copy.deepcopy(model_gpu).cpu()
    v, n, el = cpu_reference_search_conv(kind, B, S, model_cpu, 0.5 * secs, T)
    var["d_ref_arch_cpu_share"] = {"value": round(v, 1), "cores": T, "searches": n, "seconds": round(el, 2),
                                   "network": f"torch-CPU, {T} threads"}
    d = var["d_ref_arch_cpu_share"]
    loop = "mcts_ctree.py:696-827" if kind == "ez" else "mcts_ctree.py:228-321"
    return {"value": d["value"], "unit": "sims/s", "cores": T, "kind": "port",
            "sample": f"{d['searches']} full searches (B={B}, S={S}) of the reference search loop ({loop}) over the "
                      f"oracle's bit-exact ctree restatement, same conv network on torch-CPU with {T} threads, "
                      f"{d['seconds']}s; variants a-d per BASELINE.md",
            "variants": var, "host": host_cpu_info()}


def load_calibration():
    """The reference-vs-restatement timing ratios measured in the build container, where the
    reference's own ctree may run (tools/cpu_calibration.py -> profiles/cpu_calibration.json);
    the reference itself never travels to the GPU box."""
    try:
        with open(os.path.join(REPO, "profiles", "cpu_calibration.json")) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    return {k: d[k] for k in ("ref_over_port_time_tree_only", "ref_over_port_time_ref_arch", "host") if k in d}


def cpu_baseline(B, S, zero_heads, secs, device):
    """The CPU baseline of the line (rank 0, N = 1): BASELINE.md's four variants of the bit-exact
    restatement ("port"; the reference never ships to the box), each a bounded sample:
    (a) tree only, 1 thread; (b) tree only, the job's CPU share, envs partitioned;
    (c) the reference architecture with the network on this GPU (1 host thread, per-simulation
    H2D/D2H: LightZero's own deployment); (d) the reference architecture all on the CPU share.
    `value` is (d), the whole reference search loop on host cores."""
    T = share_threads()
    var = {}
    v, n, el = cpu_tree_only(B, 2, S, 1, 0.2 * secs)
    var["a_tree_only_1t"] = {"value": round(v, 1), "cores": 1, "searches": n, "seconds": round(el, 2)}
    v, n, el = cpu_tree_only(B, 2, S, T, 0.15 * secs)
    var["b_tree_only_share"] = {"value": round(v, 1), "cores": T, "searches": n, "seconds": round(el, 2)}
    model_gpu = build_model(device, zero_heads, seed=0)
    v, n, el = cpu_reference_search(B, S, model_gpu, 0.3 * secs, 1, device=device)
    var["c_ref_arch_gpu_net_1t"] = {"value": round(v, 1), "cores": 1, "searches": n, "seconds": round(el, 2),
                                    "network": "this GPU (PyTorch-ROCm), per-simulation H2D/D2H"}
    model_cpu = build_model(torch.device("cpu"), zero_heads, seed=0)
    v, n, el = cpu_reference_search(B, S, model_cpu, 0.35 * secs, T)
    var["d_ref_arch_cpu_share"] = {"value": round(v, 1), "cores": T, "searches": n, "seconds": round(el, 2),
                                   "network": f"torch-CPU, {T} threads"}
    d = var["d_ref_arch_cpu_share"]
    return {"value": d["value"], "unit": "sims/s", "cores": T, "kind": "port",
            "sample": f"{d['searches']} full searches (B={B}, S={S}) of the reference search loop "
                      f"(mcts_ctree.py:228-321) over the oracle's bit-exact ctree restatement, same MLP on "
                      f"torch-CPU with {T} threads, {d['seconds']}s; variants a-d per BASELINE.md",
            "variants": var, "host": host_cpu_info(), "calibration": load_calibration()}


BF16_PEAK_TFLOPS = 2500.0  # MI355X dense BF16 = FP16 MFMA (MI355X_MICROARCH.md: the F16 forms take the same cycles; not the 2:1-sparse figure)


def make_step(args, workload, model, device, rank):
    B, S = args.envs, args.sims
    if args.path == "fused" and args.step == "graph":
        return GraphStep(B, S, model, device, args.rng, seed=shard_seed(rank), workload=workload)
    if args.path == "fused" and args.step == "collect":
        return CollectStep(B, S, model, device, args.rng, seed=shard_seed(rank), workload=workload,
                           dst=0 if args.traj == "gather" else None)
    if workload != "cartpole":
        raise SystemExit("bench: --step python / --path generic are CartPole-only")
    return GpuStep(B, S, model, device, args.rng, args.graph, seed=shard_seed(rank), fused=args.path == "fused")


def timed_run(step, steps, warmup, world, device):
    """W untimed steps, then K timed ones between barrier + synchronize pairs; collect mode ends the
    timed region with the trajectory return. Returns (slowest rank's seconds, trajectory summary)."""
    for _ in range(warmup):
        step()
    if hasattr(step, "finish"):
        step.finish(world)  # (episodes of the warmup steps, untimed)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    # collect mode: the trajectory return ends the timed region (pack the episodes finished in
    # it on the device, return them over RCCL, sum-reduce the collector statistics)
    traj = step.finish(world) if hasattr(step, "finish") else None
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    return slowest_rank_seconds(time.perf_counter() - t0, world, device), traj


def check_step(step, S, fused):
    """every root received exactly S visits, and no search reported a broken tie-break stream
    (look-back timeout / draw-table overflow: lzm_check_errors raises)"""
    dsum = step.last[0].sum(dim=1)
    assert bool((dsum == S).all()), "visit counts do not sum to num_simulations"
    tie_errors = step.tree().check_errors()
    # fused kernels: {integrity errors, ties resolved serially, ties whose depth was published early}
    sdiag = step.tree().search_diagnostics()[:3] if fused else None
    return int(sum(tie_errors)), sdiag


L2_SHARED_ROWS_GBS_PER_CU = 70.0  # MI355X_MICROARCH.md, "Indexed rows": rows shared by every workgroup, 66-73 GB/s per CU


def conv_l2_stream_bytes(model):
    """Bytes one workgroup (one root) streams from L2 per simulation in the one-launch conv searches: every
    weight of the recurrent step — the trunk's convolutions (split-fp16: 4 B per weight), the head MLPs (f32) —
    and, for EfficientZero, its LSTM tile: the tile's K half of 64 gate columns (split-fp16 weights) and of its
    64 input rows (f32)."""
    nbytes = 0
    for net in (model.dynamics_network, model.prediction_network):
        for m in net.modules():
            if isinstance(m, (torch.nn.Conv2d, torch.nn.Linear)):
                nbytes += 4 * m.weight.numel()
    lstm = getattr(model.dynamics_network, "lstm", None)
    if lstm is not None:
        k = lstm.input_size + lstm.hidden_size
        nbytes += 2 * 64 * (k // 2) * 4
    return nbytes


def conv_roofline(step, model, B, S, device):
    """configs 5 / 3: the dominant kernel, search_conv_kernel / search_conv_ez_kernel (one launch = B x S
    simulations): the trunk's convolutions and EZ's LSTM gate GEMM run on the fp16 matrix pipe as split-fp16
    (two fp16 terms per f32 operand, three products per f32 product), so the bound is the dense
    FP16 MFMA peak (2.5 PF, as BF16) against 3x the algorithmic matrix FLOPs; the f32-equivalent rate and the
    head MLPs (VALU) ride beside."""
    ms, dbar = kernel_timing(step)
    ez = "search_conv_ez" in ms
    key, kname = ("search_conv_ez", "search_conv_ez_kernel") if ez else ("search_conv", "search_conv_kernel")
    sec = ms[key] * 1e-3
    flops, conv = conv_flops_per_sim(model, B, device)
    mfma = 3.0 * conv * B * S / sec / 1e12
    f32 = flops * B * S / sec / 1e12
    return {"bound": "mfma", "compute": "split-fp16 MFMA (v_mfma_f32_16x16x32_f16, 3 products per f32 product) "
                                        "for the conv trunk" + (" and the LSTM gate GEMM" if ez else "") +
                                        "; head MLPs on the fp32 VALU",
            "kernel": kname, "achieved": round(mfma, 2), "peak": BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(mfma / BF16_PEAK_TFLOPS, 4), "traffic": pmc_traffic(kname),
            "traffic_source": pmc_source(),
            "alg_flops_per_sim": int(flops), "alg_conv_flops_per_sim": int(conv),
            "alg_f32_tflops": round(f32, 2), "alg_f32_frac_of_fp32_peak": round(f32 / FP32_PEAK_TFLOPS, 4),
            "launch_us": round(ms[key] * 1e3, 1), "sims_per_launch": B * S,
            "mean_search_len": round(dbar, 3), "l2_stream": l2_stream(conv_l2_stream_bytes(model), S, sec)}


def l2_stream(bytes_per_sim, S, sec):
    """the L2 weight stream of one workgroup (one root per CU) against the rate the MI355X guide measured for rows
    shared by every workgroup (served by the XCD's L2): the practical bound of a stream every CU reads at once"""
    gbs = bytes_per_sim * S / sec / 1e9
    return {"bytes_per_sim_per_workgroup": int(bytes_per_sim), "achieved_GBs_per_cu": round(gbs, 1),
            "ref_GBs_per_cu": L2_SHARED_ROWS_GBS_PER_CU, "frac": round(gbs / L2_SHARED_ROWS_GBS_PER_CU, 3),
            "ref_source": "MI355X_MICROARCH.md Indexed rows: 2,048 rows shared by every workgroup, 66-73 GB/s per CU"}


def mlp_roofline(step, B, S, device):
    """config 2's dominant kernel (fused whole-search kernel: one launch = B x S simulations); its
    algorithmic work is the fp32 network (the launch is a chain of S dependent simulations,
    so neither peak bounds it; the L2 weight stream is reported beside), or, on the generic path, the
    tree kernels' HBM bytes"""
    ms, dbar = kernel_timing(step)
    if "search_mlp" in ms:
        flops = B * S * mlp_flops_per_sim(128, 2, 32, 601)
        hbm = B * (S * 8 * 128 + 2 * 32 * (1 + 2 * (S + 1)))  # latent gather+file per sim, tree slice in/out
        sec = ms["search_mlp"] * 1e-3
        achieved = flops / sec / 1e12
        R = roots_per_workgroup(B, device)
        from lightzero_amd import _lib
        resident = int(_lib.load().lzm_search_mlp_kind(B, 2, 128, 32, 601, 1)) == 1
        if resident:
            # search_res_kernel streams fc_dynamics[0] (16 slots) and the two support heads
            # (20 slots each) per simulation, slots of 256 lanes x 16 B (lzm_search_res.h)
            kname = "search_res_kernel"
            l2 = B * S * (16 + 20 + 20) * 256 * 16
        else:
            kname = "search_mlp_kernel"
            wbytes = 4 * _lib_kernel_floats()
            l2 = -(-B // R) * S * wbytes  # every workgroup streams the kernel-layout weights once per simulation
        # the network runs on the VALU (v_pk_fma_f32 chains on 1 row per workgroup: no M
        # dimension for a matrix tile), so the bound is the fp32 VALU peak and the MFMA
        # utilisation of this network step is 0 by design
        return {"bound": "valu", "compute": "fp32 VALU (v_pk_fma_f32)", "mfma_utilisation": 0.0,
                "kernel": kname, "achieved": round(achieved, 3),
                "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": round(achieved / FP32_PEAK_TFLOPS, 5),
                "traffic": pmc_traffic(kname), "traffic_source": pmc_source(), "alg_flops_per_launch": int(flops),
                "alg_hbm_bytes_per_launch": int(hbm), "hbm_achieved_GBs": round(hbm / sec / 1e9, 2),
                "l2_weight_bytes_per_launch": int(l2), "l2_achieved_TBs": round(l2 / sec / 1e12, 3),
                "l2_peak_TBs": L2_PEAK_TBS, "roots_per_workgroup": R,
                "launch_us": round(ms["search_mlp"] * 1e3, 1), "sims_per_launch": B * S,
                "mean_search_len": round(dbar, 3),
                "l2_stream": l2_stream(l2 / (-(-B // R) * S), S, sec)}
    byt = algorithmic_bytes(B, 2, 128, 601, dbar)
    dom = max(ms, key=lambda k: ms[k])
    achieved = byt[dom] / (ms[dom] * 1e-3) / 1e9
    return {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": None,
            "alg_bytes_per_launch": int(byt[dom]), "launch_us": round(ms[dom] * 1e3, 2),
            "kernels_us": {k: round(v * 1e3, 2) for k, v in ms.items()},
            "mean_search_len": round(dbar, 3)}


def workload_name(workload, B, S, world):
    if workload == "cartpole":
        return f"CartPole-v0 MuZero search, MuZeroModelMLP (latent 128, support 601), {B} envs x {S} sims per GPU"
    return (f"Breakout MuZero (BASELINE.json config 5: 2048 envs x {S} sims sharded 8x MI355X), here {world * B} envs "
            f"= {B} per GPU x {world}; conv MuZeroModel (4x64x64 frames, latent 64x8x8, support 601, 4 actions)")


def secondary_breakout(args, world, rank, device):
    """config 5 beside the headline: every rank runs the Breakout collect step on its own 256-env
    shard (BN-folded initial inference, one-launch conv search, the stand-in env's step and recording,
    one HIP graph), and the timed region ends with the trajectory return (device pack + the u8 frames and
    scalars to the learner over RCCL + statistics sum). Returns the 'config5' object."""
    B, S = args.envs, args.sims
    # enough env steps that episodes (tens of steps) finish inside the timed region and the trajectory
    # return moves real image payloads
    steps = max(args.steps, 100)
    model = build_conv_model(device, seed=0)
    step = CollectStep(B, S, model, device, args.rng, seed=shard_seed(rank), workload="breakout",
                       dst=0 if args.traj == "gather" else None)
    el, traj = timed_run(step, steps, args.warmup, world, device)
    tie_errors, sdiag = check_step(step, S, True)
    out = {"workload": workload_name("breakout", B, S, world), "step": "collect", "steps": steps,
           "value": round(whole_job_rate(B, S, steps, world, el), 1), "unit": "sims/s",
           "ms_per_step": round(el / steps * 1e3, 4), "n_gpus": world, "global_envs": world * B,
           "env_steps_per_s": round(world * B * steps / el, 1), "scaling": "weak",
           "trajectory": traj, "tie_stream_errors": tie_errors, "search_diag": sdiag,
           "data": "synthetic (random-init conv MuZeroModel; Breakout stand-in env, ALE absent)"}
    if rank == 0:
        out["roofline"] = conv_roofline(step, model, B, S, device)
        out["hbm_roofline"] = survey_hbm(out["value"] / world, 4, 4096, 601, out["roofline"]["mean_search_len"],
                                         note="per GPU (the value / n_gpus) against one GPU's HBM")
    return out


# ---------------------------------------------------------------------------------- configs 1, 3, 4
AZ_LINES = ((0, 1, 2), (3, 4, 5), (6, 7, 8), (0, 3, 6), (1, 4, 7), (2, 5, 8), (0, 4, 8), (2, 4, 6))


def az_boards(n, seed, max_moves=4):
    """config 4's synthetic positions: n TicTacToe boards, each reached by
    k ~ U{0..max_moves} random legal moves from the empty board (player 1 first), none terminal; returns
    (boards int32 [n, 9] with 0 empty / 1 / 2, start_player_index int32 [n]: 0 = player 1 to move)"""
    rng = np.random.default_rng(seed)
    boards, starts = [], []
    while len(boards) < n:
        b = np.zeros(9, np.int32)
        p = 1
        for _ in range(int(rng.integers(0, max_moves + 1))):
            b[int(rng.choice(np.flatnonzero(b == 0)))] = p
            p = 3 - p
        if any(b[i] and b[i] == b[j] == b[k] for i, j, k in AZ_LINES) or not (b == 0).any():
            continue
        boards.append(b)
        starts.append(p - 1)
    return np.stack(boards), np.asarray(starts, np.int32)


def load_calibration_key(name):
    """a reference-vs-port timing ratio measured in the build container (tools/cpu_calibration.py)"""
    try:
        with open(os.path.join(REPO, "profiles", "cpu_calibration.json")) as f:
            return json.load(f).get(name)
    except (OSError, ValueError):
        return None


def cpu_baseline_ptree(B, S, secs):
    """config 1's CPU baseline: the reference's own architecture for it — the pure-Python tree (ptree_mz.py,
    mcts_ptree.py:92-194) restated transcript-exact in oracle/ptree_port.py ("port"), MuZeroModelMLP on
    torch-CPU, 1 thread, for about `secs` (tools/ptree_bench.py)"""
    from tools.ptree_bench import run
    torch.set_num_threads(1)
    v, n, el = run(B, S, secs, False)
    cal = None
    try:
        with open(os.path.join(REPO, "profiles", "ptree_calibration.json")) as f:
            cal = {"ref_over_port_time": json.load(f)["ref_over_port_time"]}
    except (OSError, ValueError, KeyError):
        pass
    return {"value": round(v, 1), "unit": "sims/s", "cores": 1, "kind": "port",
            "sample": f"{n} searches (B={B}, S={S}) of the ptree search loop over oracle/ptree_port.py (transcript-"
                      f"exact restatement of ptree_mz.py), MuZeroModelMLP on torch-CPU, 1 thread, {el:.1f}s",
            "host": host_cpu_info(), "calibration": cal}


def cpu_baseline_az(model, boards, starts, S, secs):
    """config 4's CPU baseline: the reference AlphaZero search architecture (policy/alphazero.py:239-265,
    371-380: one tree per board, the network called per leaf, batch 1) over the bit-exact restatement of
    mcts_alphazero.cpp (oracle/az_oracle.py, "port") with the same AlphaZeroModel on torch-CPU, 1 thread,
    boards in order until about `secs`"""
    import copy
    from oracle import az_oracle
    torch.set_num_threads(1)
    net = copy.deepcopy(model).cpu().eval()
    table = az_oracle.noise_table(0.3)

    def pv(board, legal):
        b = np.asarray(board).reshape(3, 3)
        me = 1 if (b == 1).sum() == (b == 2).sum() else 2  # player 1 moved first from the empty board
        x = np.stack([(b == me), (b == 3 - me), np.full((3, 3), me)]).astype(np.float32) / 2
        with torch.no_grad():
            probs, value = net.compute_policy_value(torch.from_numpy(x).unsqueeze(0))
        p = probs.squeeze(0).numpy()
        return {int(a): float(p[a]) for a in legal}, float(value.item())

    n, t0 = 0, time.perf_counter()
    while True:
        az_oracle.search(boards[n % len(boards)], int(starts[n % len(boards)]), S, pv, True, table=table)
        n += 1
        el = time.perf_counter() - t0
        if el >= secs:
            break
    return {"value": round(n * S / el, 1), "unit": "sims/s", "cores": 1, "kind": "port",
            "sample": f"{n} board searches x {S} sims of the reference's per-board search with per-leaf network "
                      f"calls over oracle/az_oracle.py (restatement of mcts_alphazero.cpp), AlphaZeroModel on "
                      f"torch-CPU, 1 thread, {el:.1f}s",
            "host": host_cpu_info(), "calibration": load_calibration_key("az")}


def config1(args, device, cpu):
    """BASELINE.json config 1's shape (8 envs x 25 sims, CartPole MuZero MLP): the reference runs it on the
    CPU with its pure-Python tree; here the same collect-time search as the headline on the GPU"""
    B, S = 8, 25
    model = build_model(device, args.zero_heads, seed=0)
    step = GraphStep(B, S, model, device, args.rng, seed=shard_seed(0))
    steps = max(args.steps, 50)
    el, _ = timed_run(step, steps, args.warmup, 1, device)
    tie, sdiag = check_step(step, S, True)
    out = {"workload": f"CartPole-v0 MuZero (BASELINE.json config 1 shape), {B} envs x {S} sims, MuZeroModelMLP",
           "value": round(B * S * steps / el, 1), "unit": "sims/s", "ms_per_step": round(el / steps * 1e3, 4),
           "steps": steps, "n_gpus": 1, "dtype": "f32", "tie_stream_errors": tie, "search_diag": sdiag,
           "roofline": mlp_roofline(step, B, S, device)}
    out["hbm_roofline"] = survey_hbm(out["value"], 2, 128, 601, out["roofline"]["mean_search_len"])
    if cpu:
        out["cpu_baseline"] = cpu_baseline_ptree(B, S, 0.15 * args.cpu_baseline_secs)
    return out


def config3(args, device, cpu):
    """BASELINE.json config 3: Pong EfficientZero, 256 envs x 50 sims on one GPU, as the device collect step
    (efficientzero.py:538-656 inside muzero_collector.py:399-705): BN-folded conv initial inference (the
    representation network included), root preparation, the one-launch EZ search with the reward LSTM, root
    outputs, the Pong stand-in env's step and recording — one HIP graph per env step — and the timed region
    ends with the trajectory return (device packing + the process group's gather, config 5's path)"""
    B, S = args.envs, args.sims
    model = build_ez_model(device, seed=0, zero_heads=args.zero_heads)
    step = CollectStep(B, S, model, device, args.rng, seed=shard_seed(0), workload="pong",
                       dst=0 if args.traj == "gather" else None)
    steps = max(args.steps, 100)
    world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
    el, traj = timed_run(step, steps, args.warmup, world, device)
    tie, sdiag = check_step(step, S, True)
    out = {"workload": f"Atari Pong EfficientZero (BASELINE.json config 3), {B} envs x {S} sims, conv "
                       f"EfficientZeroModel (4x64x64 frames, latent 64x8x8, LSTM 512, support 101, 6 actions)",
           "step": "collect", "value": round(B * S * steps / el, 1), "unit": "sims/s",
           "ms_per_step": round(el / steps * 1e3, 4), "steps": steps, "n_gpus": 1,
           "env_steps_per_s": round(B * steps / el, 1), "trajectory": traj,
           "dtype": "f32 (convolutions as split-fp16 MFMA)",
           "search_path": step.mcts.last_path, "tie_stream_errors": tie, "search_diag": sdiag,
           "data": "synthetic (random-init conv EfficientZeroModel; Pong stand-in env, ALE absent)",
           "roofline": conv_roofline(step, model, B, S, device)}
    out["hbm_roofline"] = survey_hbm(out["value"], 6, 4096, 101, out["roofline"]["mean_search_len"], extra=4 * 512 * 4)
    if cpu:
        out["cpu_baseline"] = cpu_baseline_conv("ez", B, S, model, 0.5 * args.cpu_baseline_secs, device)
    return out


def config4(args, device, cpu):
    """BASELINE.json config 4: TicTacToe AlphaZero self-play, 512 boards x 100 sims on one GPU: the whole
    batched search (roots with the reference's noise, 100 simulations with the AlphaZeroModel in the
    kernel, the final action draw) as one lzm_az_search_fused launch per step"""
    from torch.utils.flop_counter import FlopCounterMode
    from lightzero_amd.alphazero import AlphaZeroMCTS, FusedAZNet
    from lightzero_amd.model_az import tictactoe_alphazero_model
    B, S = 512, 100
    torch.manual_seed(0)
    model = tictactoe_alphazero_model().to(device).eval()
    boards, starts = az_boards(B, 0)
    db = torch.from_numpy(boards).to(device)
    ds = torch.from_numpy(starts).to(device)
    m = AlphaZeroMCTS(9, S, 19652, 1.25, 0.3, 0.25, device=device)
    fnet = FusedAZNet(model)
    steps = max(args.steps, 20)
    with torch.no_grad():
        for _ in range(args.warmup):
            m.search_fused(db, ds, fnet, 1.0, True)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()  # (the launch stream: torch's current stream, as every lzm_* call)
        for _ in range(steps):
            m.search_fused(db, ds, fnet, 1.0, True)
        e1.record()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
    visits = m.last_visits(B)
    assert bool((visits.sum(dim=1) == S).all()), "AlphaZero root visits do not sum to num_simulations"
    with torch.no_grad():  # one more search that keeps its trees, for the mean depth
        m.search_fused(db, ds, fnet, 1.0, True, export_tree=True)
    dbar = az_mean_depth(m, B, S)
    with torch.no_grad(), FlopCounterMode(display=False) as fc:
        model.compute_policy_value(torch.zeros(B, 3, 3, 3, device=device))
    per_op = {str(k): v for k, v in fc.get_flop_counts().get("Global", {}).items()}
    flops = fc.get_total_flops() / B
    conv = sum(v for k, v in per_op.items() if "convolution" in k) / B
    sec = e0.elapsed_time(e1) * 1e-3 / steps
    ach = conv * B * S / sec / 1e12
    out = {"workload": f"TicTacToe AlphaZero self-play (BASELINE.json config 4), {B} boards x {S} sims, "
                       f"AlphaZeroModel (1 residual block x 16 channels)",
           "value": round(B * S * steps / el, 1), "unit": "sims/s", "ms_per_step": round(el / steps * 1e3, 4),
           "steps": steps, "n_gpus": 1, "dtype": "f32", "data": "synthetic (random-init AlphaZeroModel, random "
                                                                "legal positions)",
           "roofline": {"bound": "mfma", "compute": "exact f32 MFMA (v_mfma_f32_16x16x4_f32) for the convolutions, "
                                                    "heads on the VALU",
                        "kernel": "az_search_fused_kernel", "achieved": round(ach, 3), "peak": FP32_PEAK_TFLOPS,
                        "unit": "TFLOP/s", "frac": round(ach / FP32_PEAK_TFLOPS, 5),
                        "traffic": pmc_traffic("az_search_fused_kernel"), "traffic_source": pmc_source(),
                        "alg_flops_per_sim": int(flops),
                        "alg_conv_flops_per_sim": int(conv), "launch_us": round(sec * 1e6, 1),
                        "sims_per_launch": B * S},
           # the board's 27 state floats stand for the latent (gathered; the tree stores no latent to scatter)
           "hbm_roofline": survey_hbm(B * S * steps / el, 9, 27, 1, dbar, extra=4 * 9 - 4 * 27 - 8,
                                      note="AlphaZero: gather = the 27-float board state, decode = 9 policy logits + "
                                           "the value, no latent scatter")}
    if cpu:
        out["cpu_baseline"] = cpu_baseline_az(model, boards, starts, S, 0.2 * args.cpu_baseline_secs)
    return out


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}; reporting n_gpus={world}", file=sys.stderr)
    if args.dry_run:
        return dry_run(world, rank, local)
    rccl1 = None
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    elif args.rccl_world1:
        # one-rank RCCL group (a private in-memory store: no rendezvous), so the collect steps' trajectory
        # return runs the 8-GPU node's RCCL calls; the headline search has no collective in its timed region
        torch.cuda.set_device(local)
        try:
            dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1,
                                    device_id=torch.device("cuda", local))
            rccl1 = "nccl"
        except Exception as e:  # keep the headline: report the failure in the line
            rccl1 = f"failed: {type(e).__name__}: {e}"[:300]
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    if world > 1:
        ranks = [None] * world
        dist.all_gather_object(ranks, rank_info(rank, local, device))
    else:
        ranks = [rank_info(rank, local, device)]
    B, S = args.envs, args.sims
    wl = args.workload
    model = build_model(device, args.zero_heads, seed=0) if wl == "cartpole" else \
        build_conv_model(device, seed=0, zero_heads=args.zero_heads)
    step = make_step(args, wl, model, device, rank)
    el, traj = timed_run(step, args.steps, args.warmup, world, device)
    value = whole_job_rate(B, S, args.steps, world, el)
    tie_errors, sdiag = check_step(step, S, args.path == "fused")

    roofline = None
    cpu = None
    if rank == 0:
        roofline = mlp_roofline(step, B, S, device) if wl == "cartpole" else conv_roofline(step, model, B, S, device)
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(B, S, args.zero_heads, args.cpu_baseline_secs, device) if wl == "cartpole" else \
                cpu_baseline_conv("mz", B, S, model, args.cpu_baseline_secs, device)
    config5 = None
    if wl == "cartpole" and args.secondary == "breakout" and args.path == "fused":
        del step
        torch.cuda.empty_cache()
        config5 = secondary_breakout(args, world, rank, device)
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            config5["cpu_baseline"] = cpu_baseline_conv("mz", args.envs, args.sims, build_conv_model(device, seed=0),
                                                        0.5 * args.cpu_baseline_secs, device)
    extra = {}
    wanted = [c for c in args.configs.split(",") if c and c != "none"]
    if wl == "cartpole" and args.path == "fused" and world == 1:
        # the single-GPU configs of BASELINE.json beside the headline (the SCALE runs, N > 1, skip them)
        for c in wanted:
            fn = {"1": config1, "3": config3, "4": config4}[c]
            torch.cuda.empty_cache()
            extra[f"config{c}"] = fn(args, device, not args.no_cpu_baseline)
    if rank == 0:
        metric = ("MCTS simulations/sec (whole node), 256 parallel envs x 50 sims/step" if wl == "cartpole" else
                  "MCTS simulations/sec (whole node), Breakout MuZero, 256 envs per GPU x 50 sims/step")
        line = {"metric": metric,
                "value": round(value, 1), "unit": "sims/s", "n_gpus": world, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 4), "higher_is_better": True,
                "scaling": "weak", "vs_baseline": None, "dtype": "f32",
                "data": "synthetic" if wl == "cartpole" else "synthetic (random-init conv MuZeroModel, synthetic frames)",
                "config": {"workload": workload_name(wl, B, S, world),
                           "global_batch": world * B, "num_simulations": S, "rng": args.rng,
                           "path": args.path, "step": args.step if args.path == "fused" else "python",
                           "hip_graph": (args.step != "python") if args.path == "fused" else bool(args.graph),
                           "heads": "zero" if args.zero_heads else "random",
                           "parallelism": f"env-sharded x{world}"},
                "process_group": (dist.get_backend() if dist.is_initialized() else None) if rccl1 is None
                else {"world1": rccl1},
                "tie_stream_errors": tie_errors, "search_diag": sdiag, "ranks": ranks,
                "trajectory": traj, "roofline": roofline,
                "hbm_roofline": survey_hbm(value / world, 2, 128, 601, roofline["mean_search_len"],
                                           note="per GPU (the value / n_gpus) against one GPU's HBM")
                if roofline and wl == "cartpole" else
                (survey_hbm(value / world, 4, 4096, 601, roofline["mean_search_len"]) if roofline else None),
                "cpu_baseline": cpu, "config5": config5, **extra}
        print(json.dumps(line), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
