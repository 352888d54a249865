"""amp front end: opt levels O0-O5, validated option overrides, initialize, state_dict.

Reference: apex/amp/frontend.py (Properties :8-114, O3/O2/O1/O0/O4/O5 :119-247, initialize
:259-431, state_dict :434-443, load_state_dict :446-473). O4/O5 are the bf16 variants of O1/O2;
on MI355X bf16 and fp16 MFMA run at the same rate, so O5 (bf16, no loss scaling) is the
robust default and O2 (fp16 + dynamic scaling) the exact reference behaviour.
"""
from __future__ import annotations

import os
from collections import OrderedDict

import torch

from ._amp_state import _amp_state, maybe_print, warn_or_err
from ._initialize import _initialize


class Properties(object):
    """Option set with validated assignment (reference: apex/amp/frontend.py:8-114)."""

    def __init__(self):
        self.options = {
            "enabled": False,
            "opt_level": None,
            "cast_model_type": None,
            "patch_torch_functions": False,
            "patch_torch_functions_type": None,
            "keep_batchnorm_fp32": None,
            "master_weights": None,
            "loss_scale": 1.0,
        }

    def _update_options_dict(self, new_options):
        for k, v in new_options:
            if k in self.options:
                self.options[k] = v
            else:
                raise ValueError("Tried to set unexpected option {}".format(k))

    def __getattr__(self, name):
        if "options" in self.__dict__:
            options = self.__dict__["options"]
            if name in options:
                return options[name]
        raise AttributeError("'{}' object has no attribute '{}'".format(type(self).__name__, name))

    def __setattr__(self, name, value):
        if "options" not in self.__dict__ or name not in self.options:
            return super().__setattr__(name, value)
        lvl = self.opt_level
        if name == "cast_model_type":
            if lvl in {"O1", "O4"} and value is not None and value is not False and value is not torch.float32:
                warn_or_err("O1 inserts casts around Torch functions rather than model weights, so with O1, "
                            "the model weights themselves should remain FP32. If you wish to cast the model "
                            "to a different type, use opt_level='O2' or 'O3'. cast_model_type was {}".format(value))
            self.options[name] = value
        elif name == "patch_torch_functions":
            if lvl not in {"O1", "O4"} and value:
                warn_or_err("Currently, patch_torch_functions=True should only be set by selecting "
                            "opt_level='O1' or 'O4'.")
            self.options[name] = value
        elif name == "patch_torch_functions_type":
            if lvl not in {"O1", "O4"} and value is not None:
                warn_or_err("Currently, patch_torch_functions_type should only be set by selecting "
                            "opt_level='O1' or 'O4'.")
            elif lvl == "O1" and value != torch.float16:
                warn_or_err("patch_torch_functions_type should only be set to torch.float16 for opt_level='O1.")
            elif lvl == "O4" and value != torch.bfloat16:
                warn_or_err("patch_torch_functions_type should only be set to torch.bfloat16 for opt_level='O4.")
            else:
                self.options[name] = value
        elif name == "keep_batchnorm_fp32":
            if lvl in {"O1", "O4"} and value is not None:
                warn_or_err("With opt_level O1 or O4, batchnorm functions are automatically patched to run in "
                            "FP32, so keep_batchnorm_fp32 should be None. keep_batchnorm_fp32 was {}".format(value))
            if value == "False":
                self.options[name] = False
            elif value == "True":
                self.options[name] = True
            else:
                assert value is True or value is False or value is None, (
                    "keep_batchnorm_fp32 must be a boolean, the string 'True' or 'False', or None, "
                    "found keep_batchnorm_fp32={}".format(value))
                self.options[name] = value
        elif name == "master_weights":
            if lvl in {"O1", "O4"} and value is not None:
                warn_or_err("It doesn't make sense to use master_weights with O1 and O4 . With O1 and O4, "
                            "your model weights themselves should be FP32.")
            self.options[name] = value
        elif name == "loss_scale":
            self.options[name] = value if value == "dynamic" else float(value)
        else:
            self.options[name] = value


def _level(name, brief, cast, patch, patch_type, keep_bn, master, scale):
    class _L:
        def __call__(self, p):
            p.enabled = True
            p.opt_level = name
            p.cast_model_type = cast
            p.patch_torch_functions = patch
            p.patch_torch_functions_type = patch_type
            p.keep_batchnorm_fp32 = keep_bn
            p.master_weights = master
            p.loss_scale = scale
            return p

    _L.brief = brief
    _L.__name__ = name
    return _L()


opt_levels = {
    "O3": _level("O3", "O3:  Pure FP16 training.", torch.float16, False, None, False, False, 1.0),
    "O2": _level("O2", "O2:  FP16 training with FP32 batchnorm and FP32 master weights.\n",
                 torch.float16, False, None, True, True, "dynamic"),
    "O1": _level("O1", "O1:  Insert automatic casts around Pytorch functions and Tensor methods.\n",
                 None, True, torch.float16, None, None, "dynamic"),
    "O0": _level("O0", "O0:  Pure FP32 training.\n", torch.float32, False, None, None, False, 1.0),
    "O4": _level("O4", "O4:  Insert automatic casts around Pytorch functions and Tensor methods (bf16).\n",
                 None, True, torch.bfloat16, None, None, 1),
    "O5": _level("O5", "O5:  BFLOAT16 training with FP32 batchnorm and FP32 master weights.\n",
                 torch.bfloat16, False, None, True, True, 1),
}


def initialize(models, optimizers=None, enabled=True, opt_level="O1", cast_model_type=None,
               patch_torch_functions=None, patch_torch_functions_type=None, keep_batchnorm_fp32=None,
               master_weights=None, loss_scale=None, cast_model_outputs=None, num_losses=1, verbosity=1,
               min_loss_scale=None, max_loss_scale=2.0 ** 24):
    """Initialize models/optimizers for the chosen ``opt_level`` (see module docstring).

    Must be called after the model and optimizer are built and BEFORE wrapping the model in
    DistributedDataParallel. Returns the (possibly cast) model(s) and patched optimizer(s) with the
    same list/non-list structure as the inputs.
    """
    _amp_state.opt_properties = Properties()
    _amp_state.verbosity = verbosity
    if not enabled:
        return models if optimizers is None else (models, optimizers)
    if opt_level not in opt_levels:
        raise RuntimeError("Unexpected optimization level {}. Options are 'O0', 'O1', 'O2', 'O3', 'O4', 'O5'. "
                           "Note that in `O0`, `O1`, etc., the prefix O is the letter O, not the number zero."
                           .format(opt_level))
    _amp_state.opt_properties = opt_levels[opt_level](_amp_state.opt_properties)
    maybe_print("Selected optimization level {}".format(opt_levels[opt_level].brief), True)
    maybe_print("Defaults for this optimization level are:", True)
    for k, v in _amp_state.opt_properties.options.items():
        maybe_print("{:26} : {}".format(k, v), True)
    _amp_state.min_loss_scale = min_loss_scale
    _amp_state.max_loss_scale = max_loss_scale
    maybe_print("Processing user overrides (additional kwargs that are not None)...", True)
    props = _amp_state.opt_properties
    for name, val in (("enabled", enabled), ("opt_level", opt_level), ("cast_model_type", cast_model_type),
                      ("patch_torch_functions", patch_torch_functions),
                      ("patch_torch_functions_type", patch_torch_functions_type),
                      ("keep_batchnorm_fp32", keep_batchnorm_fp32), ("master_weights", master_weights),
                      ("loss_scale", loss_scale)):
        if val is not None:
            setattr(props, name, val)
    maybe_print("After processing overrides, optimization options are:", True)
    for k, v in props.options.items():
        maybe_print("{:26} : {}".format(k, v), True)
    os.environ["APEX_AMP_ENABLED"] = "1"
    return _initialize(models, optimizers, props, num_losses, cast_model_outputs)


def state_dict(destination=None):
    """``{'loss_scaler%d': {'loss_scale': float, 'unskipped': int}}`` (reference format)."""
    if destination is None:
        destination = OrderedDict()
    for idx, loss_scaler in enumerate(_amp_state.loss_scalers):
        destination["loss_scaler%d" % idx] = {
            "loss_scale": loss_scaler.loss_scale(),
            "unskipped": loss_scaler.unskipped(),
        }
    return destination


def load_state_dict(state_dict):
    if len(state_dict) != len(_amp_state.loss_scalers):
        print("Warning: state_dict contains {} entries, while {} loss_scalers are used".format(
            len(state_dict), len(_amp_state.loss_scalers)))
    state_dict = state_dict.copy()
    nb_loss_scalers = len(_amp_state.loss_scalers)
    unexpected_keys = []
    # restore by order, not by key index (reference behaviour)
    idx = 0
    for key in state_dict:
        if "loss_scaler" not in key:
            unexpected_keys.append(key)
        else:
            if idx > (nb_loss_scalers - 1):
                print("Skipping loss_scaler[{}], since num_losses was set to {}".format(idx, nb_loss_scalers))
                break
            _amp_state.loss_scalers[idx].load_scale_state(state_dict[key]["loss_scale"], state_dict[key]["unskipped"])
            idx += 1
    if len(unexpected_keys) > 0:
        raise RuntimeError("Error(s) in loading state_dict. Unexpected key(s) in state_dict: {}. ".format(
            ", ".join('"{}"'.format(k) for k in unexpected_keys)))
