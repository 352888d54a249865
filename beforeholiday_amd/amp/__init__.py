"""Automatic mixed precision (reference API: apex/amp/__init__.py:1-5)."""
from .amp import (bfloat16_function, float_function, half_function, init, promote_function,
                  register_bfloat16_function, register_float_function, register_half_function,
                  register_promote_function, deactivate)
from .handle import scale_loss, disable_casts
from .frontend import initialize, state_dict, load_state_dict, Properties, opt_levels
from ._amp_state import master_params, _amp_state
from .scaler import LossScaler

__all__ = ["init", "half_function", "bfloat16_function", "float_function", "promote_function",
           "register_half_function", "register_bfloat16_function", "register_float_function",
           "register_promote_function", "scale_loss", "disable_casts", "initialize", "state_dict",
           "load_state_dict", "master_params", "LossScaler", "deactivate"]
