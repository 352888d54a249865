"""Which form of loss * device_scale synchronises in backward (torch.cuda sync debug mode)."""
import torch

torch.cuda.set_device(0)
for name, shape_f, shape_x in [("(1,) scale x 0-dim loss", (1,), ()), ("0-dim scale x 0-dim loss", (), ()),
                               ("(1,) x (1,)", (1,), (1,))]:
    x = torch.randn(shape_x, device="cuda", requires_grad=True)
    f = torch.full(shape_f, 2.0, device="cuda")
    y = x.float() * f
    torch.cuda.synchronize()
    torch.cuda.set_sync_debug_mode("error")
    try:
        y.backward()
        torch.cuda.set_sync_debug_mode(0)
        print(name, "no sync", flush=True)
    except RuntimeError as e:
        torch.cuda.set_sync_debug_mode(0)
        print(name, "SYNC:", str(e).splitlines()[0], flush=True)
    try:
        torch.cuda.set_sync_debug_mode("error")
        z = torch.ones_like(y)
        torch.cuda.set_sync_debug_mode(0)
        print(name, "ones_like ok")
    except RuntimeError as e:
        torch.cuda.set_sync_debug_mode(0)
        print(name, "ones_like SYNC")
