"""Training checkpoint save / resume (reference workflow: README.md:63-98 — initialize amp first,
then load model / optimizer / amp state; examples/imagenet/main_amp.py save_checkpoint/--resume).

Files are written atomically (temp file + rename) and loaded with ``weights_only=True`` (no code
execution from checkpoint files)."""
import os
import tempfile

import torch


def save_checkpoint(path, model, optimizer=None, amp=None, epoch=None, extra=None):
    state = {"model": model.state_dict()}
    if optimizer is not None:
        state["optimizer"] = optimizer.state_dict()
    if amp is not None:
        state["amp"] = amp.state_dict()
    if epoch is not None:
        state["epoch"] = epoch
    if extra:
        state["extra"] = extra
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    fd, tmp = tempfile.mkstemp(dir=d, prefix="ckpt_tmp_", suffix=".pt")
    try:
        with os.fdopen(fd, "wb") as f:
            torch.save(state, f)
        os.replace(tmp, path)
    finally:
        if os.path.exists(tmp):
            os.unlink(tmp)
    return path


def load_checkpoint(path, model, optimizer=None, amp=None, map_location="cpu", strict=True):
    """Restore in the recommended order; returns the checkpoint dict (epoch / extra fields)."""
    state = torch.load(path, map_location=map_location, weights_only=True)
    model.load_state_dict(state["model"], strict=strict)
    if optimizer is not None and "optimizer" in state:
        optimizer.load_state_dict(state["optimizer"])
    if amp is not None and "amp" in state:
        amp.load_state_dict(state["amp"])
    return state
