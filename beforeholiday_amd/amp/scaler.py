"""Loss scaler (reference: apex/amp/scaler.py:42-226).

Dynamic scaling (2^16 initial, x2 after ``scale_window`` clean steps, /2 on overflow, clamped by
min/max). Unscaling of whole gradient lists is ONE multi-tensor launch (convert + scale +
overflow flag), the flag is read once per step in ``update_scale``.
"""
from __future__ import annotations

import torch

from .. import config as _config

from ..multi_tensor_apply import multi_tensor_applier
from ..ops import amp_C
from ._amp_state import maybe_print


def _has_inf_or_nan(t):
    # one host sync per tensor, like the reference's python fallback (apex/amp/scaler.py:6-21)
    v = float(t.float().sum())
    return v != v or v in (float("inf"), float("-inf"))


class LossScaler(object):
    warned_no_fused_kernel = False
    warned_unscaling_non_fp32_grad = False
    # False = the reference's "python-only install" path (per-tensor checks and copies, no
    # multi-tensor kernel); the L1 cross-product test compares both bitwise. Config.amp_python_scaler.
    has_fused_kernel = not _config.get().amp_python_scaler

    def __init__(self, loss_scale, init_scale=2.0 ** 16, scale_factor=2.0, scale_window=2000,
                 min_loss_scale=None, max_loss_scale=2.0 ** 24, device=None):
        if loss_scale == "dynamic":
            self.dynamic = True
            self._loss_scale = min(max_loss_scale, init_scale)
        else:
            self.dynamic = False
            self._loss_scale = loss_scale
        self._max_loss_scale = max_loss_scale
        self._min_loss_scale = min_loss_scale
        self._scale_seq_len = scale_window
        self._scale_factor = scale_factor
        self._unskipped = 0
        self._has_overflow = False
        if device is None:
            device = torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")
        self._overflow_buf = torch.zeros(1, dtype=torch.int, device=device)
        LossScaler.multi_tensor_scale_cuda = amp_C.multi_tensor_scale
        LossScaler.multi_tensor_axpby_cuda = amp_C.multi_tensor_axpby

    # ---- device-resident dynamic scaling (no host sync per step) ----
    # The scale and the clean-step counter live in device tensors; the overflow flag of the unscale
    # kernels is handed to the fused optimizers as their noop flag, so an overflowing step is skipped
    # ON THE DEVICE (its kernels return early) and the scale update runs as tiny device ops. The host
    # never waits for the backward to finish. FusedLAMB keeps device step counters that advance only
    # on steps the flag did not skip, so trajectories match the host path (to the rounding of fp32
    # bias corrections); the skip is not
    # printed. Enabled by Config.amp_device_scaler (bench.py) for dynamic scaling with fused optimizers.
    device_mode = False

    def enable_device_mode(self, device):
        self._scale_dev = torch.full((1,), float(self._loss_scale), dtype=torch.float32, device=device)
        self._inv_dev = torch.empty_like(self._scale_dev)
        # seeded from the host counter, so a checkpoint loaded before the first step carries over
        self._unskipped_dev = torch.full((1,), int(self._unskipped), dtype=torch.int32, device=device)
        # two flags: ``_overflow_buf`` is one backward pass's (it drives the scale update of that pass),
        # ``_step_flag`` ORs every pass since the last optimizer step and is the fused optimizers' no-op
        # flag -- an overflow in an early micro-batch of an accumulated step still skips the step
        self._overflow_buf = torch.zeros(1, dtype=torch.int, device=device)
        self._step_flag = torch.zeros(1, dtype=torch.int, device=device)
        self.device_mode = True

    def fold_pass_into_step(self):
        """Device mode: OR this pass's overflow flag into the step-level flag (one tiny kernel)."""
        torch.maximum(self._step_flag, self._overflow_buf, out=self._step_flag)

    def unskipped(self):
        return int(self._unskipped_dev.item()) if self.device_mode else self._unskipped

    def load_scale_state(self, loss_scale, unskipped):
        self._loss_scale = loss_scale
        self._unskipped = unskipped
        if self.device_mode:
            self._scale_dev.fill_(float(loss_scale))
            self._unskipped_dev.fill_(int(unskipped))

    def scale_for_loss(self):
        """The factor scale_loss multiplies the loss by: a device scalar in device mode."""
        return self._scale_dev if self.device_mode else self._loss_scale

    def loss_scale(self):
        if self.device_mode:
            return float(self._scale_dev.item())  # an explicit read: synchronises
        return self._loss_scale

    def _flag_for(self, tensors):
        # the overflow flag must live on the gradients' device
        dev = tensors[0].device
        if self._overflow_buf.device != dev:
            self._overflow_buf = torch.zeros(1, dtype=torch.int, device=dev)
        return self._overflow_buf

    def _warn_non_fp32(self, master_grads):
        if not LossScaler.warned_unscaling_non_fp32_grad and master_grads and master_grads[0].dtype != torch.float32:
            maybe_print("Attempting to unscale a grad with type {} Unscaling non-fp32 grads may indicate "
                        "an error. When using Amp, you don't need to call .half() on your model."
                        .format(master_grads[0].type()))
            LossScaler.warned_unscaling_non_fp32_grad = True

    def unscale(self, model_grads, master_grads, unused_scale, models_are_masters=False, scale_override=None):
        if self._has_overflow:
            return
        if not model_grads:
            return
        if self.device_mode and scale_override is None:
            self._warn_non_fp32(master_grads)
            torch.reciprocal(self._scale_dev, out=self._inv_dev)
            flag = self._overflow_buf
            groups = {}
            for m, s in zip(model_grads, master_grads):
                groups.setdefault((m.dtype, s.dtype), ([], []))
                groups[(m.dtype, s.dtype)][0].append(m)
                groups[(m.dtype, s.dtype)][1].append(s)
            for ins, outs in groups.values():
                multi_tensor_applier(amp_C.multi_tensor_scale, flag, [ins, outs], self._inv_dev)
            return
        scale = self._loss_scale if scale_override is None else scale_override
        if self.device_mode:
            scale = float(scale)
        if scale == 1.0 and models_are_masters and not self.dynamic:
            return
        self._warn_non_fp32(master_grads)
        if not LossScaler.has_fused_kernel:
            for m, s in zip(model_grads, master_grads):
                if m is None:
                    continue
                if self.dynamic and _has_inf_or_nan(m):
                    self._has_overflow = True
                    return
                if s is not m:
                    s.copy_(m)
                if scale != 1.0:
                    s.mul_(1.0 / scale)
            return
        # group by (model dtype, master dtype): each list passed to the kernel is single-dtype
        groups = {}
        for m, s in zip(model_grads, master_grads):
            groups.setdefault((m.dtype, s.dtype), ([], []))
            groups[(m.dtype, s.dtype)][0].append(m)
            groups[(m.dtype, s.dtype)][1].append(s)
        flag = self._flag_for(model_grads)
        for ins, outs in groups.values():
            multi_tensor_applier(LossScaler.multi_tensor_scale_cuda, flag, [ins, outs], 1.0 / scale)

    def unscale_with_stashed(self, model_grads, stashed_master_grads, master_grads, scale_override=None):
        if self._has_overflow:
            return
        grads_have_scale, stashed_have_scale, out_scale = self._loss_scale, 1.0, 1.0
        if scale_override is not None:
            grads_have_scale, stashed_have_scale, out_scale = scale_override
        if not model_grads:
            return
        self._warn_non_fp32(master_grads)
        if self.device_mode and scale_override is None:
            # the scale lives on the device: out = model_grad / scale + stashed, with the unscale
            # (and its overflow check) on the device reciprocal -- never the stale host value
            torch.reciprocal(self._scale_dev, out=self._inv_dev)
            flag = self._overflow_buf
            for m, st, out in zip(model_grads, stashed_master_grads, master_grads):
                tmp = torch.empty_like(out)
                multi_tensor_applier(amp_C.multi_tensor_scale, flag, [[m], [tmp]], self._inv_dev)
                torch.add(tmp, st, out=out)
            return
        if not LossScaler.has_fused_kernel:
            a, b = out_scale / grads_have_scale, out_scale / stashed_have_scale
            for m, st, out in zip(model_grads, stashed_master_grads, master_grads):
                if self.dynamic and _has_inf_or_nan(m):
                    self._has_overflow = True
                    return
                out.copy_(m.float() * a + st.float() * b)
            return
        groups = {}
        for m, st, out in zip(model_grads, stashed_master_grads, master_grads):
            key = (m.dtype, st.dtype, out.dtype)
            groups.setdefault(key, ([], [], []))
            for lst, t in zip(groups[key], (m, st, out)):
                lst.append(t)
        flag = self._flag_for(model_grads)
        for lists in groups.values():
            multi_tensor_applier(LossScaler.multi_tensor_axpby_cuda, flag, list(lists),
                                 out_scale / grads_have_scale, out_scale / stashed_have_scale, 0)

    def clear_overflow_state(self):
        self._has_overflow = False
        self._overflow_buf.zero_()

    def fold_and_update_device(self):
        """Device mode: ``fold_pass_into_step`` + ``update_scale`` as ONE native launch (the ~10 tiny
        torch ops they are otherwise). Returns False (never skips on the host)."""
        from .._native import available, submodule

        fn = getattr(submodule("amp_C"), "update_scale_device", None) if available() else None
        if fn is None or not self._scale_dev.is_cuda:
            self.fold_pass_into_step()
            return self.update_scale()
        fn(self._scale_dev, self._unskipped_dev, self._overflow_buf, self._step_flag, float(self._scale_factor),
           int(self._scale_seq_len), float(self._min_loss_scale or 0.0), float(self._max_loss_scale))
        return False

    def update_scale(self):
        if self.device_mode:
            # on the device: overflow -> scale / factor (>= min), counter 0; else counter + 1 and
            # scale * factor (<= max) when it reaches the window. Never skips on the host.
            ov = self._overflow_buf > 0
            down = self._scale_dev / self._scale_factor
            if self._min_loss_scale:
                down = torch.clamp(down, min=self._min_loss_scale)
            cnt = torch.where(ov, torch.zeros_like(self._unskipped_dev), self._unskipped_dev + 1)
            grow = cnt >= self._scale_seq_len
            up = torch.clamp(self._scale_dev * self._scale_factor, max=self._max_loss_scale)
            self._scale_dev.copy_(torch.where(ov, down, torch.where(grow, up, self._scale_dev)))
            self._unskipped_dev.copy_(torch.where(grow, torch.zeros_like(cnt), cnt))
            return False
        if self.dynamic and not self._has_overflow and LossScaler.has_fused_kernel:
            self._has_overflow = bool(self._overflow_buf.item())
        if self._has_overflow and self.dynamic:
            should_skip = True
            if self._min_loss_scale:
                self._loss_scale = max(self._min_loss_scale, self._loss_scale / self._scale_factor)
            else:
                self._loss_scale = self._loss_scale / self._scale_factor
            self._unskipped = 0
        else:
            should_skip = False
            self._unskipped += 1
        if self._unskipped == self._scale_seq_len and self.dynamic:
            self._loss_scale = min(self._max_loss_scale, self._loss_scale * self._scale_factor)
            self._unskipped = 0
        return should_skip


def _apply_config(c):
    # config.set(amp_python_scaler=...) / config.override take effect on the class flag too
    LossScaler.has_fused_kernel = not c.amp_python_scaler


_config.on_change(_apply_config)
