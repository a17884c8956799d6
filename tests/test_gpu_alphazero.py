"""GPU: the batched AlphaZero search (lzm_az.h through the C ABI, lightzero_amd/alphazero.py) against
the reference's own outputs (tests/golden/az_*.npz, from the compiled mcts_alphazero) and the CPU
restatement (oracle/az_oracle.py), with the float-exact scripted policy-value function on both sides.
Bar: visit counts and value sums bit-exact; action_probs (double) bit-exact."""
import glob
import os

import numpy as np
import pytest
import torch

from helpers import az_scripted_pv_torch
from oracle import az_oracle
from oracle.tictactoe import random_boards, scripted_policy_value

pytestmark = pytest.mark.gpu
GOLD = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "az_*.npz")))


def _mcts(sims, graph=False):
    from lightzero_amd.alphazero import AlphaZeroMCTS
    return AlphaZeroMCTS(9, sims, 19652, 1.25, 0.3, 0.25, device="cuda", graph=graph)


@pytest.mark.parametrize("graph", [False, True], ids=["eager", "graph"])
@pytest.mark.parametrize("path", GOLD, ids=lambda p: os.path.basename(p)[:-4])
def test_az_matches_reference_goldens(path, graph):
    g = np.load(path)
    sims, sample = int(g["sims"]), bool(g["sample"])
    m = _mcts(sims, graph)
    for _ in range(2 if graph else 1):  # graph: capture run, then a replay
        act, probs = m.get_next_actions(g["boards"], g["starts"], az_scripted_pv_torch, 1.0, sample)
        p = probs.cpu().numpy()
        assert np.array_equal(p, g["action_probs"]), np.abs(p - g["action_probs"]).max()
    v = m.last_visits(len(g["boards"])).cpu().numpy()
    assert np.array_equal(v, np.round(g["action_probs"] * sims).astype(np.int64))
    a = act.cpu().numpy()
    assert all(g["boards"][i][a[i]] == 0 for i in range(len(a)))
    if not sample:  # deterministic: first argmax
        assert np.array_equal(a, g["action_probs"].argmax(axis=1))


@pytest.mark.parametrize("max_moves,sims,sample", [(8, 60, False), (6, 150, True), (2, 400, True)])
def test_az_tree_values_match_oracle(max_moves, sims, sample):
    """deep boards (terminal positions inside the search), long searches: root children's visit
    counts and float32 value sums, and the root's own, equal the restatement's"""
    boards, starts = random_boards(24, 100 + max_moves, max_moves=max_moves)
    m = _mcts(sims)
    m.get_next_actions(boards, starts, az_scripted_pv_torch, 1.0, sample)
    visit, vsum, first, nn = [t.cpu().numpy() for t in m.export_tree(len(boards))]
    table = az_oracle.noise_table(0.3)
    for i, (b, s) in enumerate(zip(boards, starts)):
        ov, ovs, (rv, rvs) = az_oracle.search(b, int(s), sims, scripted_policy_value, sample, table=table,
                                              return_values=True)
        f = first[i, 0]
        legal = np.nonzero(b == 0)[0]
        assert f == 1 and nn[i] >= 1 + len(legal)
        gv = np.zeros(9, np.int64)
        gs = np.zeros(9, np.float32)
        gv[legal] = visit[i, f:f + len(legal)]
        gs[legal] = vsum[i, f:f + len(legal)]
        assert np.array_equal(gv, ov), (i, gv, ov)
        assert np.array_equal(gs.view(np.int32), ovs.view(np.int32)), (i, gs, ovs)
        assert visit[i, 0] == rv and vsum[i, 0].view(np.int32) == np.float32(rvs).view(np.int32)


def test_az_temperature_and_sampling():
    boards, starts = random_boards(64, 7)
    m = _mcts(40)
    act, probs = m.get_next_actions(boards, starts, az_scripted_pv_torch, 0.5, True)
    v = m.last_visits(64).cpu().numpy().astype(np.float64)
    x = v / 0.5
    ref = x / np.add.reduce(x, axis=1, keepdims=True)
    # visit_count_to_action_distribution sums in action order: compare against a sequential sum
    seq = np.zeros(64)
    for k in range(9):
        seq = seq + x[:, k]
    assert np.array_equal(probs.cpu().numpy(), x / seq[:, None])
    assert np.allclose(probs.cpu().numpy(), ref)
    a = act.cpu().numpy()
    assert all(v[i, a[i]] > 0 for i in range(64))
    # draws differ between searches (fresh Philox counter) but stay on visited actions
    a2 = m.get_next_actions(boards, starts, az_scripted_pv_torch, 0.5, True)[0].cpu().numpy()
    assert all(v[i, a2[i]] > 0 for i in range(64))


def test_az_model_batch_512():
    """C4 shape: 512 boards x 100 simulations with the restated AlphaZeroModel (random heads), graph mode"""
    from lightzero_amd.model_az import tictactoe_alphazero_model
    torch.manual_seed(0)
    net = tictactoe_alphazero_model().cuda()
    boards, starts = random_boards(512, 11)
    m = _mcts(100, graph=True)
    with torch.no_grad():
        act, probs = m.get_next_actions(boards, starts, net.compute_policy_value, 1.0, True)
        p1 = probs.clone()
        v = m.last_visits(512).cpu().numpy()
        act2, probs2 = m.get_next_actions(boards, starts, net.compute_policy_value, 1.0, True)
    assert (v.sum(axis=1) == 100).all()
    assert ((boards != 0) <= (v == 0)).all()  # no visits on occupied cells
    assert torch.equal(p1, probs2)  # same inputs, same network: the search is deterministic
    eager = _mcts(100, graph=False)
    with torch.no_grad():
        _, pe = eager.get_next_actions(boards, starts, net.compute_policy_value, 1.0, True)
    assert torch.equal(pe, p1)


def test_az_single_board_signature():
    m = _mcts(25)
    b = np.zeros(9, np.int32)
    cfg = dict(start_player_index=0, init_state=b.reshape(3, 3), katago_policy_init=False, katago_game_state=None)
    action, probs = m.get_next_action(cfg, az_scripted_pv_torch, 1.0, False)
    ref = az_oracle.search(b, 0, 25, scripted_policy_value, False)
    assert probs == list(ref / 25.0) and action == int(np.argmax(ref))


# ---------------------------------------------------------------- fused search (network inside the kernel)
def _net(seed=0, nres=1):
    from lightzero_amd.model_az import AlphaZeroModel
    torch.manual_seed(seed)
    m = AlphaZeroModel(num_res_blocks=nres, last_linear_layer_init_zero=False)
    with torch.no_grad():  # non-trivial BatchNorm statistics so the folding is exercised
        for mod in m.modules():
            if isinstance(mod, torch.nn.BatchNorm2d):
                mod.running_mean.uniform_(-0.2, 0.2)
                mod.running_var.uniform_(0.5, 1.5)
                mod.weight.uniform_(0.5, 1.5)
                mod.bias.uniform_(-0.1, 0.1)
    return m.eval().cuda()


@pytest.mark.parametrize("nres", [1, 2])
def test_fused_net_matches_torch_fp32(nres):
    """the fused network (BN folded, f32 MFMA convolutions) against the torch fp32 module; tolerance
    |d| <= 2e-5 + 2e-4 |ref| (f32, different summation order and BN folding)"""
    from lightzero_amd.alphazero import FusedAZNet
    m = _net(1, nres)
    net = FusedAZNet(m)
    boards, starts = random_boards(300, 5, max_moves=8)
    states = torch.stack([torch.from_numpy(_state(b, s)) for b, s in zip(boards, starts)]).cuda()
    torch.backends.cudnn.allow_tf32 = False
    with torch.no_grad():
        rp, rv = m.compute_policy_value(states)
        fp, fv = net.compute_policy_value(states)
    torch.testing.assert_close(fp, rp, atol=2e-5, rtol=2e-4)
    torch.testing.assert_close(fv, rv, atol=2e-5, rtol=2e-4)


def _state(board, start):
    from oracle.tictactoe import SimTicTacToe
    e = SimTicTacToe(scale=True)
    e.reset(int(start), board)
    return e.current_state()[1].astype(np.float32)


@pytest.mark.parametrize("rows", [0, 1, 2, 4, 8], ids=lambda r: f"R{r}")
@pytest.mark.parametrize("sample", [False, True], ids=["nonoise", "noise"])
def test_fused_search_equals_stepwise_search(rows, sample, monkeypatch):
    """the one-launch search against the per-simulation path fed by the same network (lzm_az_net_eval):
    identical trees (visit counts, value sums, children), action_probs and actions, bit for bit;
    ragged B (not a multiple of the boards per workgroup)"""
    from lightzero_amd.alphazero import FusedAZNet
    if rows:
        monkeypatch.setenv("LZM_AZ_BOARDS_PER_WG", str(rows))
    net = FusedAZNet(_net(2))
    boards, starts = random_boards(37, 9, max_moves=6)
    S = 30 if rows == 8 else 60  # R = 8 trees of 60 simulations do not fit in LDS
    a = _mcts(S)
    with torch.no_grad():
        act_f, pf = a.search_fused(boards, starts, net, 1.0, sample, export_tree=True)
        tf = [t.clone() for t in a.export_tree(37)]
        act_f, pf = act_f.clone(), pf.clone()
    b = _mcts(S)
    with torch.no_grad():
        act_s, ps = b.get_next_actions(boards, starts, net.compute_policy_value, 1.0, sample)
        ts = b.export_tree(37)
    assert torch.equal(pf, ps)
    assert torch.equal(act_f, act_s)
    nn = ts[3]
    assert torch.equal(tf[3], nn)
    for i in range(37):
        k = int(nn[i])
        assert torch.equal(tf[0][i, :k], ts[0][i, :k])
        assert torch.equal(tf[1][i, :k].view(torch.int32), ts[1][i, :k].view(torch.int32))
        assert torch.equal(tf[2][i, :k], ts[2][i, :k])


def test_fused_search_batch_512_properties():
    from lightzero_amd.alphazero import FusedAZNet
    net = FusedAZNet(_net(3))
    boards, starts = random_boards(512, 13)
    m = _mcts(100)
    with torch.no_grad():
        act, probs = m.search_fused(boards, starts, net, 1.0, True)
    v = m.last_visits(512).cpu().numpy()
    assert (v.sum(axis=1) == 100).all()
    assert ((boards != 0) <= (v == 0)).all()
    a = act.cpu().numpy()
    assert all(v[i, a[i]] > 0 for i in range(512))


def test_fused_rules_equal_reference_scans():
    """the fused search's stone-mask done / winner against get_done_winner's cell scan (lzm_az.h, the
    reference's order) on every one of the 3^9 boards, legal or not, and its DPP argmax of order-preserving
    score keys against the first strict maximum of a scan, on scores with ties, -inf lanes and signed zeros"""
    from lightzero_amd._lib import call, ptr, stream_ptr
    grid = np.array(np.meshgrid(*[np.arange(3)] * 9, indexing="ij")).reshape(9, -1).T.astype(np.int32)
    n = len(grid)
    rng = np.random.default_rng(3)
    sc = rng.normal(size=(n, 16)) * 10.0 ** rng.integers(-3, 3, size=(n, 1))
    k = rng.integers(0, 16, size=n)
    sc[np.arange(n), k] = sc.max(axis=1)                     # a tie with the maximum
    sc[rng.random((n, 16)) < 0.2] = -np.inf                  # lanes past the children
    z = rng.random(n) < 0.05
    sc[z] = 0.0
    sc[z, ::2] = -0.0                                        # all-zero rows: +0 / -0 are equal scores
    sc[0] = -np.inf                                          # (no child: lane 0)
    boards = torch.from_numpy(grid).cuda()
    scores = torch.from_numpy(np.ascontiguousarray(sc)).cuda()
    out = torch.zeros((n, 6), dtype=torch.int32, device="cuda")
    call("lzm_debug_az_rules", n, ptr(boards), ptr(scores), ptr(out), stream_ptr())
    o = out.cpu().numpy()
    assert np.array_equal(o[:, 0], o[:, 2]) and np.array_equal(o[:, 1], o[:, 3])
    assert (o[:, 1] != -1).sum() > 1000 and o[:, 0].sum() > 1000  # (wins and full boards occur)
    assert np.array_equal(o[:, 4], o[:, 5])
    assert np.array_equal(o[:, 5], np.argmax(sc, axis=1))       # numpy's argmax: the first maximum too
