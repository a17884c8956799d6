"""Drop-in for ``lzero.mcts.ctree.ctree_efficientzero.ez_tree`` (ez_tree.pyx:6-121), GPU-backed."""
from ._tree_api import (MinMaxStatsList, ResultsWrapper, _RootsBase, _backprop, _backprop_with_reuse, _require_list,
                        _traverse, _traverse_with_reuse)

__all__ = ["MinMaxStatsList", "ResultsWrapper", "Roots", "batch_traverse", "batch_backpropagate",
           "batch_traverse_with_reuse", "batch_backpropagate_with_reuse"]


class Roots(_RootsBase):
    EZ = True


def batch_traverse(roots, pb_c_base, pb_c_init, discount_factor, min_max_stats_lst, results, virtual_to_play_batch):
    """ez_tree.pyx:108-114."""
    return _traverse(roots, pb_c_base, pb_c_init, discount_factor, min_max_stats_lst, results, virtual_to_play_batch)


def batch_backpropagate(current_latent_state_index, discount_factor, value_prefixs, values, policies,
                        min_max_stats_lst, results, is_reset_list, to_play_batch):
    """ez_tree.pyx:83-93 (is_reset_list: 1 where the parent's value prefix restarts)."""
    _require_list("is_reset_list", is_reset_list)
    _backprop(current_latent_state_index, discount_factor, value_prefixs, values, policies, min_max_stats_lst,
              results, to_play_batch, is_reset_list)


def batch_traverse_with_reuse(roots, pb_c_base, pb_c_init, discount_factor, min_max_stats_lst, results,
                              virtual_to_play_batch, true_action, reuse_value):
    """ez_tree.pyx:116-121 (ReZero): x = -1 where the walk stopped on the expanded true-action child."""
    return _traverse_with_reuse(roots, pb_c_base, pb_c_init, discount_factor, min_max_stats_lst, results,
                                virtual_to_play_batch, true_action, reuse_value)


def batch_backpropagate_with_reuse(current_latent_state_index, discount_factor, value_prefixs, values, policies,
                                   min_max_stats_lst, results, is_reset_list, to_play_batch, no_inference_lst,
                                   reuse_lst, reuse_value_lst):
    """ez_tree.pyx:95-105 (ReZero). is_reset_list: one flag per env (see _backprop_with_reuse: the
    reference's compacted list is read by env index, undefined once an env skips inference)."""
    _require_list("is_reset_list", is_reset_list)
    _backprop_with_reuse(current_latent_state_index, discount_factor, value_prefixs, values, policies,
                         min_max_stats_lst, results, to_play_batch, no_inference_lst, reuse_lst, reuse_value_lst,
                         is_reset_list)
