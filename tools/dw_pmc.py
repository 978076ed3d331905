"""fc1-shape dW GEMM (M_out=2048, N=512, K=16384, MN-contiguous operands, split 8), register-staged
128x128 tile (wide=0) then LDS-DMA 256x128 tile (wide=1): a short fixed workload for PMC passes."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "genomics-lm_amd"))
import torch  # noqa: E402
from codonlm_amd import _lib as L, ops  # noqa: E402

M, N, K = 16384, 2048, 512
g = torch.Generator().manual_seed(0)
x = torch.randn(M, K, generator=g).to("cuda", torch.bfloat16)
dy = torch.randn(M, N, generator=g).to("cuda", torch.bfloat16)
dw = torch.empty(N, K, dtype=torch.float32, device="cuda")
for wide in (0, 1):
    L.lib.cg_gemm_set_wide(wide)
    for _ in range(5):
        ops.gemm(dy, x, a_kcontig=False, b_kcontig=False, M=N, N=K, K=M, out=dw, split_k=8)
    torch.cuda.synchronize()
L.lib.cg_gemm_set_wide(-1)
print("done")
