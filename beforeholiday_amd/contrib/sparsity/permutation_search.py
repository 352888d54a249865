"""Input-channel permutation search for 2:4 sparsity (reference:
apex/contrib/sparsity/permutation_search_kernels/call_permutation_search_kernels.py:5-74,
exhaustive_search.py:312 (stripe groups of 8 columns), permutation_utilities.py:40-93
(sum_after_2_to_4, try_swap)).

Goal: find a column permutation ``perm`` of a weight matrix ``W [R, C]`` (C = input channels,
grouped in stripes of 4) maximising the magnitude kept by 2:4 pruning of ``W[:, perm]``.

Search ("exhaustive", stripe groups of 8 = stripe pairs):

1. score EVERY stripe pair in one launch: the best of the 35 ways to regroup the pair's 8 columns
   into two stripes (``permutation_search_cuda.stripe_pair_gains``, kernels/sparsity.hip);
2. greedily apply the disjoint improving pairs, best first; repeat until no pair improves;
3. escape local optima: perturb with random cross-stripe swaps and re-converge, keep the best.

"progressive channel swap" evaluates batches of random single-column swaps until a time limit.
GPU matrices run on the HIP kernels (hard error if the extension is missing); CPU matrices use the
vectorised PyTorch scorer below (also the numerics oracle of the kernel tests).
"""
import itertools
import time

import numpy as np
import torch

from ..._native import submodule

# split k: bit j set => column j of the pair's 8 columns lands in the first stripe (column 0 always
# does); index 0 is the current layout. Same table as kernels/sparsity.hip.
SPLIT_MASKS = sorted(1 | sum(1 << k for k in c) for c in itertools.combinations(range(1, 8), 3))
# column order of the 8 columns after applying split k: first 4 -> stripe i, last 4 -> stripe j
SPLIT_ORDER = torch.tensor([[j for j in range(8) if m >> j & 1] + [j for j in range(8) if not m >> j & 1]
                            for m in SPLIT_MASKS], dtype=torch.long)


def _as_matrix(matrix):
    if isinstance(matrix, np.ndarray):
        matrix = torch.from_numpy(matrix)
    return matrix.float().contiguous()


def sum_after_2_to_4(matrix) -> float:
    """Sum of |m| kept when each row's groups of 4 consecutive columns keep their 2 largest."""
    m = _as_matrix(matrix)
    if m.is_cuda:
        return float(submodule("permutation_search_cuda").sum_after_2_to_4(m))
    R, C = m.shape
    return float(m.abs().view(R, C // 4, 4).topk(2, dim=-1).values.sum(dtype=torch.float64))


def _pair_gains_ref(m, pairs, budget_elems=1 << 25):
    R = m.shape[0]
    a = m.abs()
    P = pairs.shape[0]
    gains = torch.zeros(P, dtype=torch.float32)
    splits = torch.zeros(P, dtype=torch.int32)
    order = SPLIT_ORDER.to(m.device)
    chunk = max(1, budget_elems // max(1, R * 35 * 8))
    for s in range(0, P, chunk):
        pr = pairs[s:s + chunk].long()
        cols = torch.cat([pr[:, :1] * 4 + torch.arange(4), pr[:, 1:] * 4 + torch.arange(4)], dim=1)  # [Pc, 8]
        x = a[:, cols]                                       # [R, Pc, 8]
        x = x[:, :, order]                                   # [R, Pc, 35, 8]
        v = x.view(R, -1, 35, 2, 4).topk(2, dim=-1).values.sum(dim=(-1, -2)).sum(0)  # [Pc, 35]
        g = v - v[:, :1]
        best, idx = g[:, 1:].max(dim=1)
        pos = best > 0
        gains[s:s + chunk] = torch.where(pos, best, torch.zeros_like(best))
        splits[s:s + chunk] = torch.where(pos, idx + 1, torch.zeros_like(idx)).int()
    return gains, splits


def stripe_pair_gains(matrix, pairs):
    """(gain [P], split [P]) for stripe pairs ``pairs [P, 2]`` (see module docstring)."""
    m = _as_matrix(matrix)
    if m.is_cuda:
        return submodule("permutation_search_cuda").stripe_pair_gains(m, pairs.to(m.device, torch.int32).contiguous())
    return _pair_gains_ref(m, pairs)


def _all_pairs(S, device):
    i, j = torch.triu_indices(S, S, offset=1)
    return torch.stack([i, j], dim=1).to(device=device, dtype=torch.int32).contiguous()


def _converge(m, perm, pairs, max_pairs, gen, rel_tol=1e-7, max_iters=10000):
    C = m.shape[1]
    order = SPLIT_ORDER
    for _ in range(max_iters):
        cand = pairs
        if max_pairs is not None and pairs.shape[0] > max_pairs:
            sel = torch.randperm(pairs.shape[0], generator=gen)[:max_pairs].to(pairs.device)
            cand = pairs[sel]
        gain, split = stripe_pair_gains(m, cand)
        thr = rel_tol * max(float(m.abs().sum()), 1e-30) / max(1, C // 4)
        good = (gain > thr).nonzero().flatten()
        if good.numel() == 0:
            return m, perm
        good = good[torch.argsort(gain[good], descending=True)]
        chosen_pairs = cand[good].cpu().tolist()
        chosen_split = split[good].cpu().tolist()
        used = set()
        cols = torch.arange(C)
        for (i, j), s in zip(chosen_pairs, chosen_split):
            if i in used or j in used:
                continue
            used.update((i, j))
            eight = torch.cat([torch.arange(4 * i, 4 * i + 4), torch.arange(4 * j, 4 * j + 4)])
            new = eight[order[s]]
            cols[4 * i:4 * i + 4] = new[:4]
            cols[4 * j:4 * j + 4] = new[4:]
        m = m[:, cols.to(m.device)].contiguous()
        perm = perm[cols]
    return m, perm


def exhaustive_search(matrix, stripe_group_size=8, escape_attempts=100, max_pairs=None, seed=1,
                      perturb_swaps=None):
    """Stripe-pair regrouping search; returns ``perm`` (LongTensor [C]) with ``matrix[:, perm]`` the
    improved layout. ``stripe_group_size`` other than 8 is accepted for API parity (pairs of stripes
    are always used). On CPU ``max_pairs`` (default 4096) samples the candidate pairs per sweep."""
    del stripe_group_size
    m = _as_matrix(matrix)
    R, C = m.shape
    perm = torch.arange(C)
    if C % 4 != 0 or C < 8:
        return perm
    if max_pairs is None and not m.is_cuda:
        max_pairs = 4096
    gen = torch.Generator().manual_seed(seed)
    pairs = _all_pairs(C // 4, m.device)
    m, perm = _converge(m, perm, pairs, max_pairs, gen)
    best_m, best_perm, best_val = m, perm, sum_after_2_to_4(m)
    nswap = perturb_swaps or max(1, C // 64)
    for _ in range(escape_attempts):
        cols = torch.arange(C)
        for _ in range(nswap):
            a, b = torch.randint(0, C, (2,), generator=gen).tolist()
            if a // 4 != b // 4:
                cols[[a, b]] = cols[[b, a]]
        m2, p2 = _converge(best_m[:, cols.to(m.device)].contiguous(), best_perm[cols], pairs, max_pairs, gen)
        v2 = sum_after_2_to_4(m2)
        if v2 > best_val * (1 + 1e-7):
            best_m, best_perm, best_val = m2, p2, v2
    return best_perm


def progressive_channel_swap(matrix, time_limit=60.0, improvement_threshold=1e-9, batch=256, seed=1):
    """Random cross-stripe single-column swaps, accepted when they raise the kept magnitude, until
    ``time_limit`` seconds pass (reference: call_permutation_search_kernels.py:47-62)."""
    m = _as_matrix(matrix)
    R, C = m.shape
    perm = torch.arange(C)
    if C % 4 != 0 or C < 8:
        return perm
    gen = torch.Generator().manual_seed(seed)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < time_limit:
        src = torch.randint(0, C, (batch,), generator=gen)
        dst = torch.randint(0, C, (batch,), generator=gen)
        keep = (src // 4) != (dst // 4)
        src, dst = src[keep], dst[keep]
        if src.numel() == 0:
            continue
        # score each swap on its two stripes only
        sa, sb = (src // 4), (dst // 4)
        a = m.abs()
        ga = a[:, (sa.unsqueeze(1) * 4 + torch.arange(4)).to(m.device)]   # [R, B, 4]
        gb = a[:, (sb.unsqueeze(1) * 4 + torch.arange(4)).to(m.device)]
        before = ga.topk(2, -1).values.sum((-1, 0)) + gb.topk(2, -1).values.sum((-1, 0))
        ia, ib = (src % 4).to(m.device), (dst % 4).to(m.device)
        na, nb = ga.clone(), gb.clone()
        ar = torch.arange(src.numel(), device=m.device)
        na[:, ar, ia] = gb[:, ar, ib]
        nb[:, ar, ib] = ga[:, ar, ia]
        after = na.topk(2, -1).values.sum((-1, 0)) + nb.topk(2, -1).values.sum((-1, 0))
        imp = (after - before).cpu()
        used = set()
        cols = torch.arange(C)
        for k in torch.argsort(imp, descending=True).tolist():
            if imp[k] <= improvement_threshold:
                break
            s_, d_ = int(sa[k]), int(sb[k])
            if s_ in used or d_ in used:
                continue
            used.update((s_, d_))
            x, y = int(src[k]), int(dst[k])
            cols[[x, y]] = cols[[y, x]]
        if used:
            m = m[:, cols.to(m.device)].contiguous()
            perm = perm[cols]
    return perm


def accelerated_search_for_good_permutation(matrix_group, options=None):
    """Strategy dispatcher (reference: call_permutation_search_kernels.py:5-74). ``options``:
    ``strategy`` in {"exhaustive", "progressive channel swap", "user defined"} and the per-strategy
    keys (``stripe_group_size``, ``escape_attempts``, ``progressive_search_time_limit``,
    ``improvement_threshold``). Returns the permutation as a python list."""
    options = dict(options or {})
    strategy = options.get("strategy", "exhaustive")
    C = matrix_group.shape[1]
    if strategy == "exhaustive":
        perm = exhaustive_search(matrix_group, options.get("stripe_group_size", 8), options.get("escape_attempts", 100),
                                 max_pairs=options.get("max_pairs"))
    elif strategy == "progressive channel swap":
        perm = progressive_channel_swap(matrix_group, options.get("progressive_search_time_limit", 60),
                                        options.get("improvement_threshold", 1e-9))
    else:
        perm = torch.arange(C)
    return [int(v) for v in perm]
