"""Forward linear (NT) probe: own MFMA GEMM (gemm.mm_nt) vs F.linear (hipBLASLt) at GPT-2 / BERT shapes incl. the LM head."""
import sys, torch, json
sys.path.insert(0, ".")
from beforeholiday_amd._native import submodule
gm = submodule("gemm")
def t_ms(fn, reps=20):
    for _ in range(3): fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); s.record()
    for _ in range(reps): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / reps
for M, N, K in [(8192, 50304, 1024), (8192, 3072, 1024), (8192, 1024, 1024), (8192, 4096, 1024), (8192, 1024, 4096)]:
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
    tl = t_ms(lambda: torch.nn.functional.linear(a, b))
    to = t_ms(lambda: gm.mm_nt(a, b))
    print(json.dumps({"M": M, "N": N, "K": K, "blaslt_ms": round(tl, 4), "own_ms": round(to, 4), "speedup": round(tl / to, 3)}))
