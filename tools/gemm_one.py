"""Run a few C4-shaped GEMMs (for PMC counter passes): fwd (NT), dX (NN) and dW (TN, split-K)."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "genomics-lm_amd"))
import torch
from codonlm_amd import _lib as L, ops
M = 16384
g = torch.Generator().manual_seed(0)
for name, N, K in [("proj", 512, 512), ("fc1", 2048, 512)]:
    x = torch.randn(M, K, generator=g).to("cuda", torch.bfloat16)
    w = (torch.randn(N, K, generator=g) * 0.05).to("cuda", torch.bfloat16)
    out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    for _ in range(5):
        ops.gemm(x, w, out=out)
    # dX = dY . W  (W is [N][K] -> MN-contiguous B operand)
    dy = torch.randn(M, N, generator=g).to("cuda", torch.bfloat16)
    dx = torch.empty(M, K, dtype=torch.bfloat16, device="cuda")
    for _ in range(5):
        ops.gemm(dy, w, b_kcontig=False, M=M, N=K, K=N, out=dx)
    # dW = dY^T . X  (both MN-contiguous), fp32 out, split-K 4
    dw = torch.empty(N, K, dtype=torch.float32, device="cuda")
    for _ in range(5):
        ops.gemm(dy, x, a_kcontig=False, b_kcontig=False, M=N, N=K, K=M, out=dw, split_k=4)
torch.cuda.synchronize()
print("ok")
