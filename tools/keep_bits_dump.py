"""Dump the attention forward's keep bits and output for one C4-shaped layer (B=2) to a .npz, so two
library builds can be compared bit for bit:  CG_LIB_PATH=<lib> python tools/keep_bits_dump.py out.npz"""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "genomics-lm_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from codonlm_amd import ops  # noqa: E402

B, H, T, hd = 2, 8, 1024, 64
g = torch.Generator().manual_seed(0)
qkv = (torch.randn(B * T, 3 * H * hd, generator=g) * 0.5).to("cuda", torch.bfloat16)
idx = torch.randint(4, 68, (B, T), generator=g)
seg = ops.segment_starts(idx.to("cuda"), 3)
y, lse, mask = ops.attn_fwd_keep(qkv, seg, B, T, H, H, hd, 5, 0.1)
ref = ops.attn_drop_mask(B, T, H, 5, 0.1, "cuda")
torch.cuda.synchronize()
np.savez(sys.argv[1], y=y.float().cpu().numpy(), mask=mask.cpu().numpy(), ref=ref.cpu().numpy())
print("saved", sys.argv[1])
