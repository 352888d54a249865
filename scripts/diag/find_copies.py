"""Which aten ops of the ResNet-50 bench step launch copy / elementwise kernels (torch.profiler with
shapes): prints aten::copy_ / contiguous / add_ / clone events of one eager step with their shapes."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch.nn.functional as F
    from beforeholiday_amd import amp
    from beforeholiday_amd.models import resnet50_fused
    from beforeholiday_amd.optimizers import FusedLAMB
    from beforeholiday_amd.utils import gemm_tuning

    os.environ["BH_AMP_DEVICE_SCALER"] = "1"
    gemm_tuning.setup("auto")
    model = resnet50_fused().cuda().to(memory_format=torch.channels_last)
    opt = FusedLAMB(model.parameters(), lr=1e-3)
    model, opt = amp.initialize(model, opt, opt_level="O2", keep_batchnorm_fp32=True, verbosity=0)
    x = torch.randn(256, 3, 224, 224, device="cuda", dtype=torch.half).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (256,), device="cuda")

    def step():
        loss = F.cross_entropy(model(x), y)
        with amp.scale_loss(loss, opt) as s:
            s.backward()
        opt.step()
        opt.zero_grad()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CPU], record_shapes=True, with_stack=True) as prof:
        step()
        torch.cuda.synchronize()
    for ev in prof.events():
        if ev.name in ("aten::copy_", "aten::contiguous", "aten::add_", "aten::clone", "aten::add", "aten::mul",
                       "aten::fill_", "aten::zero_", "aten::zeros", "aten::_to_copy"):
            stack = [s for s in (ev.stack or []) if "beforeholiday_amd" in s or "bench" in s][:3]
            print(ev.name, ev.input_shapes[:2], " | ", " <- ".join(stack))


if __name__ == "__main__":
    main()
