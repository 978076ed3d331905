"""Run-to-run determinism of the bf16 MFMA attention forward / backward (p=0, hash dropout, keep-bit mask) at hd 64/48/32."""
import sys
import torch
root = sys.argv[1] if len(sys.argv) > 1 else "."
sys.path.insert(0, root + "/genomics-lm_amd")
from codonlm_amd import ops

for (B, T, H, KV, hd) in [(2, 1024, 8, 8, 64), (2, 512, 8, 4, 48), (2, 256, 4, 4, 32)]:
    g = torch.Generator().manual_seed(hd + T)
    N = (H + 2 * KV) * hd
    qkv = torch.randn(B * T, N, generator=g).to(torch.bfloat16).to("cuda")
    idx = torch.randint(4, 68, (B, T), generator=g)
    seg = ops.segment_starts(idx.to("cuda"), 3)
    mask = ops.attn_drop_mask(B, T, H, 7, 0.1, "cuda")
    res = []
    for p, m in ((0.0, None), (0.1, None), (0.1, mask)):
        outs = [ops.attn_fwd(qkv, seg, B, T, H, KV, hd, drop_seed=7, drop_p=p, drop_mask=m) for _ in range(3)]
        det = all(torch.equal(outs[0][0], o[0]) and torch.equal(outs[0][1], o[1]) for o in outs[1:])
        dy = torch.randn_like(outs[0][0])
        bw = [ops.attn_bwd(qkv, seg, outs[0][0], dy, outs[0][1], B, T, H, KV, hd, drop_seed=7, drop_p=p, drop_mask=m)
              for _ in range(3)]
        bdet = all(torch.equal(bw[0], b) for b in bw[1:])
        res.append(f"p={p} mask={m is not None}: fwd det {det} bwd det {bdet}")
    print(hd, T, " | ".join(res))
