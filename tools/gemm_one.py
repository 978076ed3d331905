"""One C4 persistent-GEMM product, a few launches per kernel, for rocprofv3 --pmc passes.

    GEMM_ONE="fc1f" python tools/gemm_one.py     (fc1f: fc1 forward plain, fc1dx: fc1 dX plain)
Kernels run in order: the eight-wave persistent kernel (CG_TILE_PERS), the loader-wave one
(CG_TILE_PERS_LW); each kernel name in the counter CSV tells them apart.
"""
import os
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "genomics-lm_amd"))
import torch  # noqa: E402
from codonlm_amd import _lib as L, ops  # noqa: E402

M, D = 16384, 512
shape = os.environ.get("GEMM_ONE", "fc1f")
N, K = {"fc1f": (4 * D, D), "fc1dx": (D, 4 * D), "qkvdx": (D, 3 * D)}[shape]
g = torch.Generator().manual_seed(0)
a = torch.randn(M, K, generator=g).to("cuda", torch.bfloat16)
b = (torch.randn(N, K, generator=g) * K ** -0.5).to("cuda", torch.bfloat16)
o = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
for tile in (L.TILE_PERS, L.TILE_PERS_LW):
    for _ in range(3):
        ops.gemm(a, b, out=o, tile=tile)
torch.cuda.synchronize()
print("ok")
