"""Driver for rocprofv3 counter passes over the transposed-operand weight-gradient GEMM (kernels/gemm_tn.hip):
the four BERT-large / GPT-2 8192-token weight-gradient shapes, the auto split count, a few calls each (the
kernel + its k_tn_reduce), fp16."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from beforeholiday_amd._native import submodule

    gm = submodule("gemm")
    T = 8192
    for n, k in ((3072, 1024), (1024, 1024), (4096, 1024), (1024, 4096)):
        dy = torch.randn(T, n, device="cuda", dtype=torch.float16)
        x = torch.randn(T, k, device="cuda", dtype=torch.float16)
        for _ in range(4):
            gm.weight_grad_tn(dy, x, 0)
        torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()
