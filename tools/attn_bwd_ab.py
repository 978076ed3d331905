"""Same-box timing of the bf16 attention backward: split (dQ kernel + dK/dV kernel) against the
fused pass (cg_attn_bwd_algo), at the benchmarked geometries (bench.py CONFIGS: batch per GPU,
dropout 0.1 from the forward's keep words, SEP segments, the q/k/v bias partials, RoPE tables for
C3).  HIP events around 20 calls after 5 warm-up calls, interleaved rounds; one JSON line per
(config, algo, round).

    python tools/attn_bwd_ab.py [c4 c3 c5 c2] [--rounds N]
"""
import argparse
import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "genomics-lm_amd"))
from codonlm_amd import _lib as L  # noqa: E402
from codonlm_amd import ops  # noqa: E402

GEOM = {  # B, T, H, KV, hd, rope
    "c4": (32, 1024, 8, 8, 64, False),
    "c3": (256, 512, 8, 4, 48, True),
    "c5": (128, 512, 8, 8, 48, False),
    "c2": (256, 512, 4, 4, 64, False),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="*", default=["c4", "c3", "c5", "c2"])
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--n", type=int, default=20)
    a = ap.parse_args()
    st = torch.cuda.current_stream().cuda_stream
    for name in a.configs:
        B, T, H, KV, hd, rope = GEOM[name]
        p, seed = 0.1, 77
        N = (H + 2 * KV) * hd
        g = torch.Generator().manual_seed(1)
        qkv = (torch.randn(B * T, N, generator=g) * 0.5).to("cuda", torch.bfloat16)
        dy = torch.randn(B * T, H * hd, generator=g).to("cuda", torch.bfloat16)
        idx = torch.randint(4, 68, (B, T), generator=g)
        idx[:, T // 3] = 3
        seg = ops.segment_starts(idx.to("cuda"), 3)
        y, lse, mask = ops.attn_fwd_keep(qkv, seg, B, T, H, KV, hd, seed, p)
        dqkv = torch.zeros_like(qkv)
        part = torch.empty(B * ((T + 127) // 128), N, dtype=torch.float32, device="cuda")
        ws = torch.empty(int(L.lib.cg_attn_bwd_workspace(B, T, H)) // 4 + 1, dtype=torch.float32, device="cuda")
        rc = rs = None
        if rope:
            half = hd // 2
            inv = 1.0 / (10000 ** (torch.arange(half, dtype=torch.float64) / half))
            ang = torch.arange(T, dtype=torch.float64)[:, None] * inv[None, :]
            rc, rs = torch.cos(ang).float().cuda(), torch.sin(ang).float().cuda()

        def call(algo):
            L.check(L.lib.cg_attn_bwd_algo(
                algo, 1, qkv.data_ptr(), N, seg.data_ptr(), y.data_ptr(), H * hd,
                dy.data_ptr(), H * hd, lse.data_ptr(), dqkv.data_ptr(), N, B, T, H, KV, hd, 0, seed, p,
                mask.data_ptr(), part.data_ptr(), N, rc.data_ptr() if rope else None,
                rs.data_ptr() if rope else None, ws.data_ptr(), ws.numel() * 4, st), "cg_attn_bwd_algo")

        for r in range(a.rounds):
            for algo, an in ((1, "split"), (2, "fused")):
                for _ in range(5):
                    call(algo)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.n):
                    call(algo)
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1000 / a.n
                print(json.dumps({"config": name, "algo": an, "round": r, "us_per_layer": round(us, 1)}), flush=True)


if __name__ == "__main__":
    main()
