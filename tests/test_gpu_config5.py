"""GPU: config 5's per-rank path — the Breakout MuZero collect step (BASELINE.json config 5, SURVEY.md
§8(e)): BN-folded conv initial inference, the one-launch conv search in collect-step mode, the Atari
stand-in env (lzm_atari.h), device episode packing (lzm_episodes_*) and the image trajectory blocks.

Env parity is unpinned (ALE absent; the env is a stand-in with Breakout's action set and frame format):
the device env is checked against its numpy restatement (oracle/breakout_synth.py), which re-derives
every recorded frame and reward from an episode's first frame and actions. The search is checked
bit-exactly against the same search driven call by call; the device packing against the torch
restatement of the layout (trajectory.pack_episodes).
"""
import numpy as np
import pytest
import torch

import bench
from oracle import breakout_synth

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


def _conv_model(seed=0):
    return bench.build_conv_model(DEV, seed=seed)


def _collector(n=32, S=8, T=120, E=8, seed=3, graph=True, record_pred=False, model=None):
    from lightzero_amd.collector import DeviceCollector
    return DeviceCollector(model or _conv_model(), n, S, device=DEV, seed=seed, graph=graph, poll_every=4,
                           episode_slots=E, max_episode_steps=T, env="breakout", record_pred=record_pred)


def test_breakout_episodes_replay_through_the_restated_game():
    col = _collector()
    blocks, stats = col.collect_blocks(n_episode=24, to_host=True)
    (b,) = blocks
    assert b.frames.dtype == np.uint8 and b.frames.shape[1:] == (1, 64, 64)
    assert stats["episodes"] == b.num_episodes >= 24
    for env_id, L, r0 in b.index:
        sc = b.scalars[r0:r0 + L + 1]
        fr = b.frames[r0:r0 + L + 1]
        actions, rewards = np.rint(sc[:L, 0]).astype(np.int64), sc[:L, 1]
        assert 1 <= L <= col.T and set(np.unique(actions)) <= {0, 1, 2, 3}
        assert set(np.unique(rewards)) <= {0.0, 1.0}  # ClipRewardWrapper
        assert (sc[:L, 2:6].sum(axis=1) == col.S).all()  # root visit counts of an S-simulation search
        # row L: zeros but for the reward column, the episode's unclipped score (eval_episode_return)
        assert sc[L, 0] == 0 and (sc[L, 2:] == 0).all() and sc[L, 1] >= rewards.sum()
        msg = breakout_synth.replay_episode(fr, actions, rewards, col.T, episode_return=sc[L, 1])
        assert msg is None, f"env {env_id} episode of {L} steps: {msg}"


def test_breakout_collect_unpacks_to_reference_frames():
    """collect() returns GameSegment-shaped dicts: float32 frames in [0, 1] (frame / 255, the
    wrappers' ScaledFloatFrame) of shape (1, 64, 64), one per step plus the final one"""
    col = _collector(n=16, seed=5)
    eps, stats = col.collect(n_episode=16)
    assert len(eps) >= 16
    for e in eps:
        L = len(e["action_segment"])
        assert e["obs_segment"].shape == (L + 1, 1, 64, 64) and e["obs_segment"].dtype == np.float32
        assert e["obs_segment"].max() <= 1.0 and e["obs_segment"].min() >= 0.0
        u8 = np.rint(e["obs_segment"] * 255).astype(np.uint8)
        np.testing.assert_allclose(u8.astype(np.float32) / 255.0, e["obs_segment"], rtol=0, atol=1e-7)
        np.testing.assert_allclose(e["child_visit_segment"].sum(1), 1.0, atol=1e-6)


@pytest.mark.parametrize("env", ["cartpole", "breakout"])
def test_device_pack_equals_torch_pack(env):
    """lzm_episodes_scan / lzm_episodes_pack == trajectory.pack_episodes (the layout's restatement)
    on the same recorded slots, including the predicted-value column"""
    from lightzero_amd.collector import DeviceCollector
    from lightzero_amd.trajectory import pack_episodes
    from tests.test_gpu_collect import _model
    model = _model() if env == "cartpole" else _conv_model()
    col = DeviceCollector(model, 24, 8, device=DEV, seed=11, graph=True, poll_every=4, episode_slots=6,
                          max_episode_steps=100, env=env, record_pred=True)
    for rnd in range(3):
        for _ in range(12):
            col.step()
        counts = col.ep_count.cpu().numpy().astype(np.int64)
        ln = col.ep_len.cpu().numpy()
        todo = [(i, k % col.E, int(ln[i, k % col.E])) for i in range(col.n) for k in range(int(col._consumed[i]),
                                                                                        int(counts[i]))]
        ref = pack_episodes(col.rec_frames, col.rec_action, col.rec_reward, col.rec_visits, col.rec_value, todo,
                            col.rec_pred, col.env.frame_scale, ep_return=col.ep_return)
        got = col.pack_new()
        assert got.num_episodes == len(todo)
        np.testing.assert_array_equal(got.index.cpu().numpy(), ref.index.numpy())
        assert torch.equal(got.frames, ref.frames)
        assert torch.equal(got.scalars, ref.scalars)
        np.testing.assert_array_equal(col._consumed, counts)
    assert col.pack_new().num_episodes == 0  # nothing new since the last pack


def test_pack_detects_overwritten_slots():
    col = _collector(n=8, S=4, T=40, E=2, seed=1)
    for _ in range(200):  # > 2 episodes of <= 40 steps per env: the slots wrap before any pack
        col.step()
    with pytest.raises(RuntimeError, match="overwritten"):
        col.pack_new()


def test_conv_collect_step_search_equals_plain_search():
    """the one-launch conv search in collect-step mode (device seeds from the step counter, root
    outputs, fresh min-max bounds) equals MuZeroMCTSCtree.search called with the same seeds"""
    from lightzero_amd.collect import DeviceSearchStep
    from lightzero_amd.mcts_ctree import MuZeroMCTSCtree
    from lightzero_amd.utils import EasyDict
    B, S, seed = 64, 20, 4
    model = _conv_model()
    rng = np.random.default_rng(seed)
    obs = torch.from_numpy(bench.synthetic_obs("breakout", B, rng)).to(DEV)
    noises = torch.from_numpy(rng.dirichlet([0.3] * 4, size=B).astype(np.float32)).to(DEV)
    step = DeviceSearchStep(model, B, S, [list(range(4))] * B, (4, 64, 64), DEV, seed=seed, graph=False)
    step.set_inputs(obs=obs, noises=noises)
    outs = []
    for _ in range(2):
        o = step.step()
        outs.append((o["distributions"].clone(), o["values"].clone()))
    assert step.mcts.last_path == "fused-conv"
    cfg = EasyDict(dict(num_simulations=S, discount_factor=0.997, device=DEV,
                        model=dict(support_scale=300, categorical_distribution=True)))
    mcts = MuZeroMCTSCtree(cfg)
    base = (1000003 * seed) % 1000000
    with torch.no_grad():
        for n, (dist, vals) in enumerate(outs):
            out = step.initial.initial_inference(obs)
            roots = MuZeroMCTSCtree.roots(B, [list(range(4))] * B)
            roots.prepare_device(0.25, noises, torch.zeros(B, device=DEV), out.policy_logits,
                                 torch.full((B,), -1, dtype=torch.int32, device=DEV))
            seeds = torch.tensor([(base + n * S + k) % 1000000 for k in range(S)], dtype=torch.int32, device=DEV)
            mcts.search(roots, model, out.latent_state, torch.full((B,), -1, dtype=torch.int32, device=DEV),
                        seeds=seeds)
            assert mcts.last_path == "fused-conv"
            assert torch.equal(roots.tree.distributions(), dist)
            assert torch.equal(roots.tree.values(), vals)
            roots.clear()


def test_breakout_graph_step_equals_eager():
    from lightzero_amd.collector import DeviceCollector
    n, S = 16, 8
    model = _conv_model()
    out = []
    for graph in (True, False):
        col = DeviceCollector(model, n, S, device=DEV, seed=9, graph=graph, poll_every=2, episode_slots=4,
                              max_episode_steps=100, env="breakout")
        for _ in range(12):
            col.step()
        torch.cuda.synchronize()
        out.append((col.rec_action.cpu().numpy(), col.rec_visits.cpu().numpy(), col.env.state.cpu().numpy(),
                    col.rec_frames.cpu().numpy()))
    for a, b in zip(out[0], out[1]):
        np.testing.assert_array_equal(a, b)


def test_folded_initial_inference_matches_module_on_gpu():
    """the BN-folded representation + prediction (conv_infer.FoldedConvInitial) vs the module, f32
    tolerance, on the GPU (MIOpen convolutions with the lzm_bias_add_relu epilogue, the 8 x 8 tail on
    the split-bf16 trunk, lzm_conv_resnet8_p) for both conv families"""
    from lightzero_amd.conv_infer import FoldedConvInitial
    from lightzero_amd.model_conv import atari_efficientzero_model
    torch.manual_seed(1)
    ez = atari_efficientzero_model(last_linear_layer_init_zero=False)
    bench._random_bn(ez, 2)
    for m in (_conv_model(), ez.to(DEV).eval()):
        obs = torch.rand(32, 4, 64, 64, device=DEV)
        with torch.no_grad():
            ref = m.initial_inference(obs)
            got = FoldedConvInitial(m).initial_inference(obs)
        for k in ("latent_state", "value", "policy_logits"):
            torch.testing.assert_close(getattr(got, k), getattr(ref, k), rtol=1e-4, atol=1e-5)


def test_bench_breakout_workload_line(tmp_path):
    """`bench.py --workload breakout` (config 5's per-GPU shard) prints one line with the conv roofline"""
    import json
    import os
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--workload", "breakout", "--steps", "2",
                        "--warmup", "1", "--envs", "32", "--sims", "8", "--no-cpu-baseline", "--step", "collect"],
                       capture_output=True, text=True, timeout=240, cwd=repo)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert "Breakout MuZero" in line["config"]["workload"] and line["value"] > 0
    assert line["roofline"]["kernel"] == "search_conv_kernel" and line["roofline"]["bound"] == "mfma"
    assert line["tie_stream_errors"] == 0 and line["trajectory"]["frame_dtype"] == "uint8"


@pytest.mark.parametrize("kind,B,cin", [("mz", 37, 4), ("ez", 37, 4), ("mz", 300, 4), ("mz", 45, 3), ("mz", 29, 7)])
def test_native_downsample_matches_float64_reference(kind, B, cin):
    """lzm_repr_downsample (the DownSample stages on split-bf16 MFMA, csrc/lzm_repr.h) vs the same BN-folded
    convolutions in float64 on the CPU: conv 3x3/2 -> 32, the 32-channel block, the downsample block with its
    3x3/2 shortcut, the 64-channel block, avg pool. B = 37: tiles of several images per workgroup, a ragged last
    round; B = 300: ~10 tiles per workgroup, every slot of the LDS-DMA ring reused several times; 3 and 7
    observation planes: the first layer's im2col over other channel counts. Three launches must agree bit for
    bit (a DMA read before it lands would show as run-to-run differences). Tolerance: the two-term fp16 split
    keeps f32-level error — 2e-5 of the layer's magnitude (relative to max |ref|); the achieved ratio is
    printed."""
    import torch.nn.functional as F
    from lightzero_amd.conv_infer import FoldedConvInitial
    from lightzero_amd.model_conv import atari_efficientzero_model, atari_muzero_model
    if kind == "mz" and cin == 4:
        m = _conv_model(4)
    elif kind == "mz":
        torch.manual_seed(cin)
        m = atari_muzero_model(observation_shape=(cin, 64, 64), last_linear_layer_init_zero=False)
        bench._random_bn(m, cin + 1)
        m = m.to(DEV).eval()
    else:
        torch.manual_seed(4)
        m = atari_efficientzero_model(last_linear_layer_init_zero=False)
        bench._random_bn(m, 5)
        m = m.to(DEV).eval()
    fi = FoldedConvInitial(m)
    assert fi.repr_native is not None
    obs = torch.rand(B, cin, 64, 64, device=DEV)
    with torch.no_grad():
        runs = [fi._downsample_native(obs).cpu() for _ in range(3)]
    for r in runs[1:]:
        assert torch.equal(r, runs[0])
    got = runs[0].double()
    x = obs.cpu().double()
    ops = [tuple(t.cpu().double() if torch.is_tensor(t) else t for t in op) for op in fi.ops[:fi.tail[0]]]
    for op in ops:
        if op[0] == "conv_relu":
            x = F.conv2d(x, op[1], op[2], stride=op[3], padding=1).relu()
        elif op[0] == "basic":
            y = F.conv2d(x, op[1], op[2], padding=1).relu()
            x = (F.conv2d(y, op[3], op[4], padding=1) + x).relu()
        elif op[0] == "down":
            y = F.conv2d(x, op[1], op[2], stride=2, padding=1).relu()
            x = (F.conv2d(y, op[3], op[4], padding=1) + F.conv2d(x, op[5], None, stride=2, padding=1)).relu()
        else:
            x = F.avg_pool2d(x, 3, 2, 1)
    assert got.shape == x.shape == (B, 64, 8, 8)
    err = (got - x).abs()
    print(f"downsample {kind} B={B} C={cin}: max |err| / max |ref| = {float(err.max() / x.abs().max()):.3e}")
    assert float(err.max()) <= 2e-5 * float(x.abs().max()), float(err.max() / x.abs().max())
    torch.testing.assert_close(got, x, rtol=1e-4, atol=2e-5 * float(x.abs().max()))
