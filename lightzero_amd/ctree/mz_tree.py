"""Drop-in for ``lzero.mcts.ctree.ctree_muzero.mz_tree`` (mz_tree.pyx:5-107), GPU-backed."""
from ._tree_api import (MinMaxStatsList, ResultsWrapper, _backprop, _backprop_with_reuse, _RootsBase, _traverse,
                        _traverse_with_reuse)

__all__ = ["MinMaxStatsList", "ResultsWrapper", "Roots", "batch_traverse", "batch_backpropagate",
           "batch_traverse_with_reuse", "batch_backpropagate_with_reuse"]


class Roots(_RootsBase):
    EZ = False


def batch_traverse(roots, pb_c_base, pb_c_init, discount_factor, min_max_stats_lst, results, virtual_to_play_batch):
    """mz_tree.pyx:95-101 -> (latent_state_index_in_search_path, latent_state_index_in_batch,
    last_actions, virtual_to_play_batchs)."""
    return _traverse(roots, pb_c_base, pb_c_init, discount_factor, min_max_stats_lst, results, virtual_to_play_batch)


def batch_backpropagate(current_latent_state_index, discount_factor, value_prefixs, values, policies,
                        min_max_stats_lst, results, to_play_batch):
    """mz_tree.pyx:74-80."""
    _backprop(current_latent_state_index, discount_factor, value_prefixs, values, policies, min_max_stats_lst,
              results, to_play_batch)


def batch_traverse_with_reuse(roots, pb_c_base, pb_c_init, discount_factor, min_max_stats_lst, results,
                              virtual_to_play_batch, true_action, reuse_value):
    """mz_tree.pyx:102-107 (ReZero): x = -1 where the walk stopped on the expanded true-action child."""
    return _traverse_with_reuse(roots, pb_c_base, pb_c_init, discount_factor, min_max_stats_lst, results,
                                virtual_to_play_batch, true_action, reuse_value)


def batch_backpropagate_with_reuse(current_latent_state_index, discount_factor, value_prefixs, values, policies,
                                   min_max_stats_lst, results, to_play_batch, no_inference_lst, reuse_lst,
                                   reuse_value_lst):
    """mz_tree.pyx:84-93 (ReZero)."""
    _backprop_with_reuse(current_latent_state_index, discount_factor, value_prefixs, values, policies,
                         min_max_stats_lst, results, to_play_batch, no_inference_lst, reuse_lst, reuse_value_lst)
