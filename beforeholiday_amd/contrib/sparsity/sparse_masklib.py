"""Structured (m:n) sparsity masks (reference: apex/contrib/sparsity/sparse_masklib.py:9-184).

The masks match the 2:4 layout consumed by CDNA4's sparse MFMA (``v_smfmac``): along the reduction
(input-channel) dimension, every group of m=4 consecutive weights keeps the n=2 of largest magnitude.
All searches are vectorised tensor ops (one matmul against the table of valid patterns), no loops
over groups.
"""
import sys
from itertools import permutations

import torch


def fill(x):
    return float(x.nonzero().size(0)) / torch.numel(x)


def reshape_1d(matrix, m):
    """[rows, cols] -> [rows * ceil(cols/m), m] (zero padded)."""
    if matrix.shape[1] % m > 0:
        pad = torch.zeros(matrix.shape[0], matrix.shape[1] + (m - matrix.shape[1] % m), dtype=matrix.dtype,
                          device=matrix.device)
        pad[:, :matrix.shape[1]] = matrix
        return pad.view(-1, m), pad.shape
    return matrix.view(-1, m), matrix.shape


_valid_1d = {}


def compute_valid_1d_patterns(m, n):
    key = (m, n)
    if key not in _valid_1d:
        base = [1] * n + [0] * (m - n)
        pats = sorted(set(permutations(base)))
        _valid_1d[key] = torch.tensor(pats, dtype=torch.float32)
    return _valid_1d[key]


def mn_1d_best(matrix, m, n):
    """Keep, in every group of m along a row, the n entries maximising the kept |magnitude|."""
    patterns = compute_valid_1d_patterns(m, n).to(matrix.device)
    mask = torch.ones_like(matrix, dtype=torch.float32)
    mat, shape = reshape_1d(matrix.abs().float(), m)
    pmax = torch.argmax(mat @ patterns.t(), dim=1)
    mask = patterns[pmax].view(shape)[:, :matrix.shape[1]]
    return mask.view(matrix.shape)


def m4n2_1d(mat, density):
    return mn_1d_best(mat, 4, 2)


def mn_2d_greedy(matrix, m, n):
    """m x m blocks, greedily keep largest entries while every row and column keeps <= n."""
    mat = matrix.abs().float().cpu()
    R, C = mat.shape
    mask = torch.ones(R, C)
    for r0 in range(0, R - R % m, m):
        for c0 in range(0, C - C % m, m):
            blk = mat[r0:r0 + m, c0:c0 + m]
            keep = torch.zeros(m, m)
            rows = [0] * m
            cols = [0] * m
            for idx in torch.argsort(blk.flatten(), descending=True).tolist():
                r, c = divmod(idx, m)
                if rows[r] < n and cols[c] < n:
                    keep[r, c] = 1
                    rows[r] += 1
                    cols[c] += 1
            mask[r0:r0 + m, c0:c0 + m] = keep
    return mask.to(matrix.device)


def m4n2_2d_greedy(mat, density):
    return mn_2d_greedy(mat, 4, 2)


_valid_2d = {}


def compute_valid_2d_patterns(m, n):
    key = (m, n)
    if key not in _valid_2d:
        rows = compute_valid_1d_patterns(m, n)
        import itertools
        pats = []
        for combo in itertools.product(range(rows.size(0)), repeat=m):
            p = rows[list(combo)]
            if (p.sum(0) <= n).all():
                pats.append(p)
        _valid_2d[key] = torch.stack(pats)
    return _valid_2d[key]


def mn_2d_best(matrix, m, n):
    """m x m blocks: the valid (row- and column-n:m) pattern maximising kept |magnitude|."""
    patterns = compute_valid_2d_patterns(m, n).to(matrix.device)  # [P, m, m]
    R, C = matrix.shape
    mask = torch.ones(R, C, device=matrix.device)
    Rm, Cm = R - R % m, C - C % m
    if Rm and Cm:
        blocks = matrix[:Rm, :Cm].abs().float().view(Rm // m, m, Cm // m, m).permute(0, 2, 1, 3).reshape(-1, m * m)
        best = torch.argmax(blocks @ patterns.view(-1, m * m).t(), dim=1)
        chosen = patterns[best].view(Rm // m, Cm // m, m, m).permute(0, 2, 1, 3).reshape(Rm, Cm)
        mask[:Rm, :Cm] = chosen
    return mask


def m4n2_2d_best(mat, density):
    return mn_2d_best(mat, 4, 2)


def create_mask(tensor, pattern="m4n2_1d", density=0.5):
    """Mask with the tensor's shape and dtype. 4-D conv weights [K, C, R, S] are pruned along C."""
    shape = tensor.shape
    t = tensor.float().contiguous()
    func = getattr(sys.modules[__name__], pattern, None)
    if func is None:
        raise ValueError(f"unknown sparsity pattern {pattern}")
    if len(shape) == 1:
        mask = func(t.view(1, shape[0]), density)
    elif len(shape) == 2:
        mask = func(t, density)
    elif len(shape) == 3:
        mask = func(t.view(shape[0] * shape[1], shape[2]), density)
    elif len(shape) == 4:
        tt = t.permute(2, 3, 0, 1).contiguous().view(shape[2] * shape[3] * shape[0], shape[1])
        mask = func(tt, density).view(shape[2], shape[3], shape[0], shape[1]).permute(2, 3, 0, 1).contiguous()
    else:
        raise ValueError("unsupported tensor rank for sparsity")
    return mask.view(shape).to(tensor.dtype)
