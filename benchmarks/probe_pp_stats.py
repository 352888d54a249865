"""Kernel-time probe for rocprofv3 (scripts/prof_one.sh): the ping-pong GEMM (tile mode 4) with and
without its BatchNorm-statistics epilogue at two ResNet-50 1x1 shapes, 10 launches each."""
import os, sys, torch
sys.path.insert(0, os.getcwd())
from beforeholiday_amd._native import submodule
from beforeholiday_amd.ops import conv_bn
gm = submodule("gemm"); gm.set_force_mfma(True); gm.set_tile_mode(4)
for M, N, K in [(200704, 512, 128), (50176, 1024, 256)]:
    a = torch.randn(M, K, device="cuda", dtype=torch.float16)
    b = torch.randn(N, K, device="cuda", dtype=torch.float16) * 0.05
    ks = torch.zeros(N, device="cuda")
    for _ in range(10):
        gm.linear_act(a, b, None, 0, False)
    for _ in range(10):
        conv_bn.gemm_bn(a, b, "stats", kshift=ks)
    torch.cuda.synchronize()
