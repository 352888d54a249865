from .asp import ASP
from .permutation_lib import Permutation
from .permutation_search import (accelerated_search_for_good_permutation, exhaustive_search, progressive_channel_swap,
                                 stripe_pair_gains, sum_after_2_to_4)
from .sparse_masklib import create_mask

__all__ = ["ASP", "Permutation", "create_mask", "accelerated_search_for_good_permutation", "exhaustive_search",
           "progressive_channel_swap", "stripe_pair_gains", "sum_after_2_to_4"]
