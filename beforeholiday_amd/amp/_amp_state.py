"""Global amp state shared by the amp modules (reference: apex/amp/_amp_state.py)."""
import torch


class AmpState(object):
    def __init__(self):
        self.hard_override = False
        self.allow_incoming_model_not_fp32 = False
        self.verbosity = 1
        self.opt_properties = None
        self.loss_scalers = []
        self.handle = None
        self.min_loss_scale = None
        self.max_loss_scale = 2.0 ** 24


_amp_state = AmpState()


def warn_or_err(msg):
    if _amp_state.hard_override:
        print("Warning:  " + msg)
    else:
        raise RuntimeError(msg)


def _distributed():
    return (torch.distributed.is_available() and torch.distributed.is_initialized()
            and torch.distributed.get_world_size() > 1)


def maybe_print(msg, rank0=False):
    if _amp_state.verbosity > 0:
        if rank0 and _distributed():
            if torch.distributed.get_rank() == 0:
                print(msg)
        else:
            print(msg)


def master_params(optimizer):
    """Iterates over the params owned by ``optimizer`` (the fp32 masters under O2). A pending fused
    mixed-precision step first materialises the master gradients, so e.g. gradient clipping on them
    sees what the unfused path would have produced."""
    plan = getattr(getattr(optimizer, "_amp_stash", None), "plan", None)
    if plan is not None and hasattr(plan, "materialize"):
        plan.materialize()
    for group in optimizer.param_groups:
        for p in group["params"]:
            yield p
