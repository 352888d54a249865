"""Legacy fp16 utilities (reference API: apex/fp16_utils/__init__.py:1-16)."""
from .fp16util import (BN_convert_float, network_to_half, prep_param_lists, model_grads_to_master_grads,
                       master_params_to_model_params, tofp16, to_python_float, clip_grad_norm, convert_module,
                       convert_network, FP16Model)
from .fp16_optimizer import FP16_Optimizer
from .loss_scaler import LossScaler, DynamicLossScaler
