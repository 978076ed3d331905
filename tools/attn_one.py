"""One forward + backward of the C4 attention (dropout 0.1, SEP segments), for PMC passes.
Uses the engine's path: keep bits written by the forward (cg_attn_fwd_keep); ATTN_MASK=1: made by
cg_attn_drop_mask first (the round-2 path), ATTN_HASH=1: hashed in every kernel.  The backward runs
once per algorithm (split: dQ + dK/dV kernels; fused: attn_bwd_fused_mfma), so one PMC pass counts both."""
import os
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "genomics-lm_amd"))
import torch
from codonlm_amd import ops

B, H, T, hd = int(os.environ.get("ATTN_B", "32")), 8, 1024, 64  # ATTN_B: the bench's B (32 since round 5)
g = torch.Generator().manual_seed(0)
qkv = (torch.randn(B * T, 3 * H * hd, generator=g) * 0.5).to("cuda", torch.bfloat16)
idx = torch.randint(4, 68, (B, T), generator=g)
seg = ops.segment_starts(idx.to("cuda"), 3)
hashed = os.environ.get("ATTN_HASH") == "1"
separate = os.environ.get("ATTN_MASK") == "1"
for _ in range(2):
    if hashed or separate:
        mask = None if hashed else ops.attn_drop_mask(B, T, H, 5, 0.1, "cuda")
        y, lse = ops.attn_fwd(qkv, seg, B, T, H, H, hd, drop_seed=5, drop_p=0.1, drop_mask=mask)
    else:
        y, lse, mask = ops.attn_fwd_keep(qkv, seg, B, T, H, H, hd, 5, 0.1)
    dy = torch.randn_like(y)
    for algo in ("split", "fused"):
        if algo == "fused" and mask is None:
            continue
        ops.attn_bwd(qkv, seg, y, dy, lse, B, T, H, H, hd, drop_seed=5, drop_p=0.1, drop_mask=mask, algo=algo)
torch.cuda.synchronize()
print("ok")
