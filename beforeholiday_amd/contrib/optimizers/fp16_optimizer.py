"""FP16_Optimizer for the legacy contrib fused optimizers (reference:
apex/contrib/optimizers/fp16_optimizer.py:4-240): fp32 master copies, static or dynamic loss
scale, overflow check via the fused l2-norm's non-finite flag (one host read per step), the
fused optimizer writes the fp16 model weights in its update pass."""
import torch

from ...multi_tensor_apply import multi_tensor_applier
from ...ops import amp_C


class FP16_Optimizer(object):
    def __init__(self, init_optimizer, static_loss_scale=1.0, dynamic_loss_scale=False, dynamic_loss_args=None,
                 verbose=True):
        self.optimizer = init_optimizer
        self.fp16_groups = []
        self.fp32_groups = []
        for group in self.optimizer.param_groups:
            f16 = list(group["params"])
            f32 = [p.detach().clone().float() for p in f16]
            self.fp16_groups.append(f16)
            self.fp32_groups.append(f32)
            group["params"] = f32
        dev = self.fp16_groups[0][0].device if self.fp16_groups and self.fp16_groups[0] else torch.device("cpu")
        self.overflow_buf = torch.zeros(1, dtype=torch.int, device=dev)
        if dynamic_loss_scale:
            if dynamic_loss_args is not None:
                raise SystemError("Do not support dynamic loss scale args for now.")
            self.dynamic_loss_scale = True
            self.cur_scale = 2 ** 16
            self.cur_iter = 0
            self.last_overflow_iter = -1
            self.scale_factor = 2
            self.scale_window = 1000
        else:
            self.dynamic_loss_scale = False
            self.cur_iter = 0
            self.cur_scale = static_loss_scale
        self.verbose = verbose

    def zero_grad(self, set_grads_to_None=True):
        from ...optimizers._common import zero_param_grads

        zero_param_grads([p for group in self.fp16_groups for p in group], set_grads_to_None)

    def step(self, closure=None):
        fp16_grads = [[p.grad for p in group] for group in self.fp16_groups]
        self.overflow_buf.zero_()
        norms = []
        for g in fp16_grads:
            if g:
                norm, _ = multi_tensor_applier(amp_C.multi_tensor_l2norm, self.overflow_buf, [g], True)
                norms.append(norm)
        if int(self.overflow_buf.item()) != 0:
            self._update_scale(True)
            return
        self.optimizer.step(grads=fp16_grads, output_params=self.fp16_groups, scale=self.cur_scale,
                            grad_norms=norms)
        self._update_scale(False)

    def backward(self, loss):
        (loss.float() * self.cur_scale).backward()

    def _update_scale(self, skip):
        if self.dynamic_loss_scale:
            if skip:
                if self.verbose:
                    print(f"\nGrad overflow on iteration {self.cur_iter}")
                    print(f"Using dynamic loss scale of {self.cur_scale}")
                self.cur_scale = max(self.cur_scale / self.scale_factor, 1)
                self.last_overflow_iter = self.cur_iter
            elif (self.cur_iter - self.last_overflow_iter) % self.scale_window == 0:
                self.cur_scale *= self.scale_factor
        elif skip:
            print("\nGrad overflow on iteration", self.cur_iter)
            print("Using static loss scale of", self.cur_scale)
        self.cur_iter += 1

    def _get_state(self):
        return self.optimizer.state

    def _set_state(self, value):
        self.optimizer.state = value

    state = property(_get_state, _set_state)

    def _get_param_groups(self):
        return self.optimizer.param_groups

    def _set_param_groups(self, value):
        self.optimizer.param_groups = value

    param_groups = property(_get_param_groups, _set_param_groups)

    def state_dict(self):
        sd = {"dynamic_loss_scale": self.dynamic_loss_scale, "cur_scale": self.cur_scale, "cur_iter": self.cur_iter,
              "optimizer_state_dict": self.optimizer.state_dict(), "fp32_groups": self.fp32_groups}
        if self.dynamic_loss_scale:
            sd.update(last_overflow_iter=self.last_overflow_iter, scale_factor=self.scale_factor,
                      scale_window=self.scale_window)
        return sd

    def load_state_dict(self, state_dict):
        self.dynamic_loss_scale = state_dict["dynamic_loss_scale"]
        self.cur_scale = state_dict["cur_scale"]
        self.cur_iter = state_dict["cur_iter"]
        if self.dynamic_loss_scale:
            self.last_overflow_iter = state_dict["last_overflow_iter"]
            self.scale_factor = state_dict["scale_factor"]
            self.scale_window = state_dict["scale_window"]
        self.optimizer.load_state_dict(state_dict["optimizer_state_dict"])
        for cur, saved in zip(self.fp32_groups, state_dict["fp32_groups"]):
            for c, s in zip(cur, saved):
                c.data.copy_(s.data)
