"""Automatic SParsity: 2:4 structured pruning workflow (reference: apex/contrib/sparsity/asp.py:18-312).

``init_model_for_pruning`` registers a boolean mask buffer per eligible weight,
``init_optimizer_for_pruning`` wraps ``optimizer.step`` to mask gradients before and weights after
the update, ``compute_sparse_masks`` computes the m:n masks (optionally stowing pruned values on the
CPU so ``restore_pruned_weights`` can undo it). With ``allow_permutation`` the first mask computation
is preceded by the offline input-channel permutation (permutation_lib.py: torch.fx channel spaces +
stripe-pair search on the HIP kernels) that raises the magnitude kept by 2:4 pruning without
changing the network function.
"""
import types

import torch

from .permutation_lib import Permutation
from .sparse_masklib import create_mask


def eligible_modules(model, whitelist_layer_types, allowed_layer_names, disallowed_layer_names):
    out = []
    for name, mod in model.named_modules():
        if isinstance(mod, whitelist_layer_types) and name not in disallowed_layer_names:
            if allowed_layer_names is not None and name not in allowed_layer_names:
                continue
            out.append((name, mod))
    return out


class ASP:
    __model = None
    __verbosity = 0
    __optimizer = None
    __sparse_parameters = []
    __calculate_mask = None
    __allow_permutation = False
    __permuted = False

    @classmethod
    def init_model_for_pruning(cls, model, mask_calculator="m4n2_1d", verbosity=3,
                               whitelist=[torch.nn.Linear, torch.nn.Conv1d, torch.nn.Conv2d, torch.nn.Conv3d],
                               allowed_layer_names=None, disallowed_layer_names=[], allow_recompute_mask=False,
                               custom_layer_dict={}, allow_permutation=True):
        assert cls.__model is None, "ASP has been initialized already."
        cls.__model = model
        cls.__verbosity = verbosity
        cls.__allow_permutation = allow_permutation
        cls.__permuted = False
        if isinstance(mask_calculator, str):
            cls.__calculate_mask = lambda p: create_mask(p, mask_calculator).bool()
        else:
            cls.__calculate_mask = mask_calculator
        sparse_parameter_list = {torch.nn.Linear: ["weight"], torch.nn.Conv1d: ["weight"],
                                 torch.nn.Conv2d: ["weight"], torch.nn.Conv3d: ["weight"]}
        whitelist = list(whitelist)
        if custom_layer_dict:
            sparse_parameter_list.update(custom_layer_dict)
            whitelist += list(custom_layer_dict.keys())
        for t in whitelist:
            assert t in sparse_parameter_list, f"Module {t} :: Don't know how to sparsify module."
        cls.__sparse_parameters = []
        for name, module in eligible_modules(model, tuple(whitelist), allowed_layer_names, disallowed_layer_names):
            names = sparse_parameter_list[type(module)]
            for p_name, p in module.named_parameters():
                if p_name not in names or not p.requires_grad:
                    continue
                if p.dtype in (torch.float32, torch.float16, torch.bfloat16) and \
                        (p.size(0) % 8 != 0 or p.size(1) % 16 != 0):
                    if verbosity >= 3:
                        print(f"[ASP] Auto skipping pruning {name}::{p_name} of size={tuple(p.size())} and "
                              f"type={p.dtype} for sparsity")
                    continue
                if verbosity >= 3:
                    print(f"[ASP] Sparsifying {name}::{p_name} of size={tuple(p.size())} and type={p.dtype}")
                mask = torch.ones_like(p, dtype=torch.bool)
                buf = p_name.split(".")[-1]
                module.register_buffer(f"__{buf}_mma_mask", mask)
                pruned = None
                if allow_recompute_mask:
                    pruned = torch.zeros_like(p, device="cpu")
                    module.register_buffer(f"__{buf}_mma_pruned_p", pruned)
                cls.__sparse_parameters.append((name, module, p_name, p, mask, pruned))

    @classmethod
    def already_init_asp_model(cls):
        return cls.__model is not None

    @classmethod
    def init_optimizer_for_pruning(cls, optimizer):
        assert cls.__optimizer is None, "ASP has initialized optimizer already."
        assert cls.__calculate_mask is not None, \
            "Called ASP.init_optimizer_for_pruning before ASP.init_model_for_pruning."
        cls.__optimizer = optimizer
        orig_step = optimizer.step

        def step(opt_self, *args, **kwargs):
            with torch.no_grad():
                for _, _, _, p, mask, _ in cls.__sparse_parameters:
                    if p.grad is not None:
                        p.grad.mul_(mask)
            rval = orig_step(*args, **kwargs)
            with torch.no_grad():
                for _, _, _, p, mask, _ in cls.__sparse_parameters:
                    p.mul_(mask)
            return rval

        optimizer.step = types.MethodType(step, optimizer)

    @classmethod
    def compute_sparse_masks(cls):
        if cls.__allow_permutation and not cls.__permuted:
            model = cls.__model.module if hasattr(cls.__model, "module") and \
                isinstance(cls.__model.module, torch.nn.Module) else cls.__model
            all_params = [(n, p) for n, p in model.named_parameters()]
            Permutation.set_permutation_params_from_asp(model, cls.__sparse_parameters, all_params, cls.__optimizer)
            Permutation.set_identical_seed()
            groups = Permutation.permute_model(model)
            cls.__permuted = True
            if cls.__verbosity >= 2 and groups is not None:
                n = sum(1 for g in groups if g.get("permutation_sequence") is not None)
                print(f"[ASP] input-channel permutation applied to {n} of {len(groups)} channel groups")
        with torch.no_grad():
            for name, module, p_name, p, mask, pruned in cls.__sparse_parameters:
                if mask.sum() < mask.numel():
                    assert pruned is not None, "Unable to restore dense parameter because allow_recompute_mask == False"
                    p.add_(pruned.to(p.device))
                mask.set_(cls.__calculate_mask(p).to(mask.device))
                if pruned is not None:
                    pruned.set_((p * (~mask)).cpu())
                p.mul_(mask)
                if cls.__verbosity >= 2:
                    print(f"[ASP] Enabled {100.0 - 100.0 * float(mask.sum()) / mask.numel():.2f}% sparsity for "
                          f"{name}::{p_name} of size={tuple(p.size())} and type={p.dtype}")

    @classmethod
    def restore_pruned_weights(cls):
        with torch.no_grad():
            for name, module, p_name, p, mask, pruned in cls.__sparse_parameters:
                if mask.sum() < mask.numel():
                    assert pruned is not None, "Unable to restore dense parameter because allow_recompute_mask == False"
                    p.add_(pruned.to(p.device))
                    mask.fill_(1)
                    pruned.zero_()

    @classmethod
    def is_sparsity_enabled(cls):
        total = sp100 = sp50 = 0
        for _, _, _, _, mask, _ in cls.__sparse_parameters:
            total += 1
            s, n = int(mask.sum()), mask.numel()
            if s == n:
                sp100 += 1
            elif 2 * s == n:
                sp50 += 1
        assert total in (sp100, sp50), "Inconsistent model sparsity"
        return total != sp100

    @classmethod
    def prune_trained_model(cls, model, optimizer):
        cls.init_model_for_pruning(model, mask_calculator="m4n2_1d", verbosity=2,
                                   whitelist=[torch.nn.Linear, torch.nn.Conv2d], allow_recompute_mask=False)
        cls.init_optimizer_for_pruning(optimizer)
        cls.compute_sparse_masks()

    @classmethod
    def set_permutation_saving_params(cls, allow_permutation=True, save_permutation_graph=False,
                                      permutation_output_dir="."):
        cls.__allow_permutation = allow_permutation
        Permutation.set_permutation_saving_params(allow_permutation, save_permutation_graph, permutation_output_dir)

    @classmethod
    def _reset(cls):
        """Forget the attached model / optimizer (tests)."""
        cls.__model = None
        cls.__optimizer = None
        cls.__sparse_parameters = []
        cls.__calculate_mask = None
        cls.__permuted = False
