"""One 4-layer grouped dW launch (C4 shapes) per tile variant, for rocprofv3 --pmc passes."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "genomics-lm_amd"))
import torch
from codonlm_amd import ops

M, d, nqkv, hid = 16384, 512, 1536, 2048
prods = []
for _ in range(4):
    for n, k in [(nqkv, d), (d, d), (hid, d), (d, hid)]:
        prods.append((torch.randn(M, n, device="cuda").to(torch.bfloat16), torch.randn(M, k, device="cuda").to(torch.bfloat16),
                      torch.empty(n, k, device="cuda"), 1.0, False))
for bm in (128, 129, 256):
    ops.gemm_dw_grouped(prods, tile_m=bm)
torch.cuda.synchronize()
print("ok")
