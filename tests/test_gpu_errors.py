"""GPU: the sticky integrity words of a tree handle (lzm_check_errors) — a broken parity-mode
tie-break stream (look-back spin timeout, draw-table overflow, LSTM hand-off timeout) must raise from
whichever result getter runs first after the search, exactly once, must not leak into the next owner
of a pooled tree, and must stop the device collector paths."""
import ctypes
import ctypes.util

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


def _poke_error(tree, word=0, value=1):
    """write `value` into sticky error word `word` of the tree's handle (hipMemcpy H2D)"""
    torch.cuda.synchronize()
    hip = ctypes.CDLL("libamdhip64.so.7" if ctypes.util.find_library("amdhip64") is None else
                      ctypes.util.find_library("amdhip64"))
    src = ctypes.c_int32(value)
    dst = tree.error_word(word)
    rc = hip.hipMemcpy(dst, ctypes.byref(src), ctypes.c_size_t(4), ctypes.c_int(1))  # hipMemcpyHostToDevice
    assert rc == 0


def _search(B=8, S=6):
    from lightzero_amd.mcts_ctree import MuZeroMCTSCtree
    from lightzero_amd.utils import EasyDict
    from tests.test_gpu_collect import _model
    model = _model()
    cfg = EasyDict(dict(num_simulations=S, discount_factor=0.997, device=DEV,
                        model=dict(support_scale=300, categorical_distribution=True)))
    mcts = MuZeroMCTSCtree(cfg)
    roots = MuZeroMCTSCtree.roots(B, [[0, 1]] * B)
    with torch.no_grad():
        out = model.initial_inference(torch.randn(B, 4, device=DEV))
    roots.prepare(0.25, [[0.5, 0.5]] * B, [0.0] * B, out.policy_logits.cpu().tolist(), [-1] * B)
    mcts.search(roots, model, out.latent_state, [-1] * B)
    return mcts, model, roots, out



@pytest.mark.parametrize("getter", ["get_distributions", "get_values", "get_trajectories"])
def test_first_getter_raises_once_and_clears(getter):
    from lightzero_amd._lib import LzmError
    _, _, roots, _ = _search()
    _poke_error(roots.tree, 0)
    with pytest.raises(LzmError):
        getattr(roots, getter)()
    # the words were cleared as they were read: the other getters of the same search do not raise again
    roots.get_distributions()
    roots.get_values()
    roots.get_trajectories()
    roots.clear()


def test_pooled_tree_does_not_carry_errors_to_next_owner():
    from lightzero_amd.mcts_ctree import MuZeroMCTSCtree
    mcts, model, roots, out = _search()
    tree = roots.tree
    _poke_error(tree, 1)  # set after the search, never read by this owner
    roots.clear()  # back to the pool with the word still set
    B = 8
    roots2 = MuZeroMCTSCtree.roots(B, [[0, 1]] * B)
    roots2.prepare(0.25, [[0.5, 0.5]] * B, [0.0] * B, out.policy_logits.cpu().tolist(), [-1] * B)
    assert roots2.tree is tree  # the pooled handle was reused
    mcts.search(roots2, model, out.latent_state, [-1] * B)
    d = roots2.get_distributions()  # a clean search does not raise
    assert all(sum(r) == 6 for r in d)
    roots2.clear()


def test_device_collector_pull_new_raises_on_error_word():
    from lightzero_amd._lib import LzmError
    from lightzero_amd.collector import DeviceCollector
    from tests.test_gpu_collect import _model
    col = DeviceCollector(_model(), 8, 6, device=DEV, seed=2, graph=True, poll_every=2)
    for _ in range(4):
        col.step()
    col.pull_new()  # clean
    _poke_error(col.search.roots.tree, 0)
    with pytest.raises(LzmError):
        col.pull_new()


def test_muzero_collector_device_path_raises_on_error_word():
    """MuZeroCollector's device path polls through DeviceCollector.pull_new, which checks the words"""
    from lightzero_amd._lib import LzmError
    from lightzero_amd.collector import DeviceCollector
    from lightzero_amd.envs import DeviceCartPoleEnvManager
    from lightzero_amd.policy import MuZeroCollectPolicy, policy_config
    from lightzero_amd.worker import MuZeroCollector
    from tests.test_gpu_muzero_collector import _model
    cfg = policy_config(num_simulations=6, game_segment_length=20, device=DEV, n_episode=8)
    collector = MuZeroCollector(env=DeviceCartPoleEnvManager(8, seed=3), policy=MuZeroCollectPolicy(cfg, _model(2)),
                                policy_config=cfg)
    orig = DeviceCollector.pull_new

    def poisoned(self):
        _poke_error(self.search.roots.tree, 2)
        return orig(self)
    DeviceCollector.pull_new = poisoned
    try:
        with pytest.raises(LzmError):
            collector.collect(n_episode=8, train_iter=0, policy_kwargs={'temperature': 1.0, 'epsilon': 0.0})
    finally:
        DeviceCollector.pull_new = orig
