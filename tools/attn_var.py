"""Attention kernel timings under variants (dropout on/off, SEP segments on/off) at C4 shape."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "genomics-lm_amd"))
import torch
from codonlm_amd import _lib as L, ops

B, H, T, hd = 16, 8, 1024, 64
g = torch.Generator().manual_seed(0)
qkv = (torch.randn(B * T, 3 * H * hd, generator=g) * 0.5).to("cuda", torch.bfloat16)
idx = torch.randint(4, 68, (B, T), generator=g)
seg = ops.segment_starts(idx.to("cuda"), 3)
tri = 2.0 * B * H * hd * T * (T + 1) / 2


def t(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / it * 1e-3


for p in (0.0, 0.1):
    for sg in (None, seg):
        y, lse = ops.attn_fwd(qkv, sg, B, T, H, H, hd, drop_seed=5, drop_p=p)
        dy = torch.randn_like(y)
        f = lambda: ops.attn_fwd(qkv, sg, B, T, H, H, hd, drop_seed=5, drop_p=p)
        bw = lambda: ops.attn_bwd(qkv, sg, y, dy, lse, B, T, H, H, hd, drop_seed=5, drop_p=p)
        a, b = t(f), t(bw)
        print(f"p={p} seg={'yes' if sg is not None else 'no '} fwd {a*1e6:7.1f}us {2*tri/a/1e12:6.1f}TF  "
              f"bwd {b*1e6:7.1f}us {7*tri/b/1e12:6.1f}TF", flush=True)
