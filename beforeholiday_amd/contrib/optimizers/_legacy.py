"""Shared helpers for the legacy (pre-AMP) contrib optimizers whose ``step`` receives gradients /
output parameters / a loss scale explicitly (reference: apex/contrib/optimizers/fused_adam.py:64-,
fused_sgd.py:115-)."""
import types


def group_lists(x, n_groups):
    """Normalise the legacy per-group argument forms (None, generator, flat list, list of lists)."""
    if x is None:
        return [None] * n_groups
    if isinstance(x, types.GeneratorType):
        return [list(x)]
    x = list(x)
    if len(x) == 0 or not isinstance(x[0], (list, tuple)):
        return [x]
    return [list(g) for g in x]
