"""Drop-in for ``lzero.mcts.ctree.ctree_efficientzero.ez_tree`` (ez_tree.pyx:6-121), GPU-backed."""
from ._tree_api import MinMaxStatsList, ResultsWrapper, _RootsBase, _backprop, _require_list, _traverse

__all__ = ["MinMaxStatsList", "ResultsWrapper", "Roots", "batch_traverse", "batch_backpropagate"]


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
