"""One C4 persistent-GEMM product, a few launches per variant, for rocprofv3 --pmc passes.

    GEMM_ONE="fc1f" python tools/gemm_one.py     (fc1f: fc1 forward plain, fc1dx: fc1 dX plain)
Variants run in order: base (loader-wave kernel), pp1 (gemm_pp.h), pp2 (gemm_pp2.h); each kernel
name in the counter CSV tells them apart.
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
for pp, pp2 in ((0, 0), (1, 0), (0, 1)):
    L.lib.cg_gemm_set_pers_pp(pp)
    L.lib.cg_gemm_set_pers_pp2(pp2)
    for _ in range(3):
        ops.gemm(a, b, out=o)
torch.cuda.synchronize()
print("ok")
