"""Same-box timing of the bf16 attention forward's dropout modes at a bench geometry: no dropout,
keep bits made by the forward itself (cg_attn_fwd_keep, DROP 3, what the engine runs), keep bits read
from a precomputed mask (cg_attn_fwd with drop_mask, DROP 2), the hash in the kernel (DROP 1), and
the mask kernel alone (cg_attn_drop_mask).  HIP events around 20 calls after 5 warm-up calls.

    python tools/attn_fwd_modes.py [c4|c3|c5|c2]
"""
import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "genomics-lm_amd"))
from codonlm_amd import ops  # noqa: E402

GEOM = {"c4": (32, 1024, 8, 8, 64), "c3": (256, 512, 8, 4, 48), "c5": (128, 512, 8, 8, 48), "c2": (256, 512, 4, 4, 64)}


def timeit(fn, n=20):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / n


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "c4"
    B, T, H, KV, hd = GEOM[name]
    g = torch.Generator().manual_seed(0)
    qkv = (torch.randn(B * T, (H + 2 * KV) * hd, generator=g) * 0.5).to("cuda", torch.bfloat16)
    idx = torch.randint(4, 68, (B, T), generator=g)
    idx[:, T // 3] = 3
    seg = ops.segment_starts(idx.to("cuda"), 3)
    p, seed = 0.1, 99
    mask = ops.attn_drop_mask(B, T, H, seed, p, "cuda")
    res = {
        "nodrop": timeit(lambda: ops.attn_fwd(qkv, seg, B, T, H, KV, hd)),
        "keep_drop3": timeit(lambda: ops.attn_fwd_keep(qkv, seg, B, T, H, KV, hd, seed, p, mask=mask)),
        "mask_drop2": timeit(lambda: ops.attn_fwd(qkv, seg, B, T, H, KV, hd, drop_seed=seed, drop_p=p, drop_mask=mask)),
        "hash_drop1": timeit(lambda: ops.attn_fwd(qkv, seg, B, T, H, KV, hd, drop_seed=seed, drop_p=p)),
        "mask_kernel": timeit(lambda: ops.attn_drop_mask(B, T, H, seed, p, "cuda")),
    }
    print(json.dumps({"config": name, **{k: round(v, 1) for k, v in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
