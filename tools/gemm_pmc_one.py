"""One GEMM shape under both tile modes (for PMC passes): dW of fc1 (both operands MN-contiguous)
and dX of fc1 (B MN-contiguous).  Usage: python tools/gemm_pmc_one.py"""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "genomics-lm_amd"))
import torch
from codonlm_amd import _lib as L, ops
M, N, K = 16384, 2048, 512
g = torch.Generator().manual_seed(0)
x = torch.randn(M, K, generator=g).to("cuda", torch.bfloat16)
w = (torch.randn(N, K, generator=g) * 0.05).to("cuda", torch.bfloat16)
dy = torch.randn(M, N, generator=g).to("cuda", torch.bfloat16)
dw = torch.empty(N, K, dtype=torch.float32, device="cuda")
dx = torch.empty(M, K, dtype=torch.bfloat16, device="cuda")
for mode in (0, 1):
    L.lib.cg_gemm_set_wide(mode)
    for _ in range(3):
        ops.gemm(dy, x, a_kcontig=False, b_kcontig=False, M=N, N=K, K=M, out=dw, split_k=8)
    for _ in range(3):
        ops.gemm(dy, w, b_kcontig=False, M=M, N=K, K=N, out=dx)
torch.cuda.synchronize()
print("ok")
