"""Same-box timing of the C4 attention kernels of one or more library builds (HIP events around
cg_attn_fwd / cg_attn_bwd, with and without the bias partials; dropout 0.1 from keep bits).

    python tools/attn_time.py [lib.so ...]     (default: the in-tree build)

Loads each library with plain ctypes (older builds lack newer symbols), so the builds compared
need only the attention entry points.  Prints one JSON line per build."""
import ctypes as C
import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
vp, i32, i64, u32, f32, sz = C.c_void_p, C.c_int, C.c_longlong, C.c_uint32, C.c_float, C.c_size_t
SIG = {
    "cg_attn_fwd": (i32, [i32, vp, i64, vp, vp, i64, vp, i32, i32, i32, i32, i32, i32, u32, f32, vp, vp]),
    "cg_attn_drop_mask_bytes": (sz, [i32, i32, i32]),
    "cg_attn_drop_mask": (i32, [i32, i32, i32, u32, f32, vp, vp]),
    "cg_attn_bwd_workspace": (sz, [i32, i32, i32]),
    "cg_attn_bwd": (i32, [i32, vp, i64, vp, vp, i64, vp, i64, vp, vp, i64, i32, i32, i32, i32, i32, i32,
                          u32, f32, vp, vp, i64, vp, sz, vp]),
}
BF16 = 1


def load(path):
    lib = C.CDLL(str(path))
    for n, (r, a) in SIG.items():
        getattr(lib, n).restype = r
        getattr(lib, n).argtypes = a
    return lib


def main():
    libs = sys.argv[1:] or [str(ROOT / "genomics-lm_amd/codonlm_amd/libcodonlm_hip.so")]
    B, H, T, hd, p, seed = 16, 8, 1024, 64, 0.1, 5
    g = torch.Generator().manual_seed(0)
    qkv = (torch.randn(B * T, 3 * H * hd, generator=g) * 0.5).to("cuda", torch.bfloat16)
    dy = (torch.randn(B * T, H * hd, generator=g)).to("cuda", torch.bfloat16)
    seg = torch.zeros(B, T, dtype=torch.int32, device="cuda")
    y = torch.empty(B * T, H * hd, dtype=torch.bfloat16, device="cuda")
    lse = torch.empty(B * H * T, dtype=torch.float32, device="cuda")
    dqkv = torch.zeros_like(qkv)
    bpart = torch.empty(B * ((T + 127) // 128), 3 * H * hd, dtype=torch.float32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    for path in libs:
        lib = load(path)
        mask = torch.empty(int(lib.cg_attn_drop_mask_bytes(B, T, H)) // 4 + 1, dtype=torch.int32, device="cuda")
        ws = torch.empty(int(lib.cg_attn_bwd_workspace(B, T, H)) // 4 + 1, dtype=torch.float32, device="cuda")

        def fwd():
            assert lib.cg_attn_fwd(BF16, qkv.data_ptr(), qkv.stride(0), seg.data_ptr(), y.data_ptr(), y.stride(0),
                                   lse.data_ptr(), B, T, H, H, hd, 0, seed, p, mask.data_ptr(), st) == 0

        def bwd(bp):
            assert lib.cg_attn_bwd(BF16, qkv.data_ptr(), qkv.stride(0), seg.data_ptr(), y.data_ptr(), y.stride(0),
                                   dy.data_ptr(), dy.stride(0), lse.data_ptr(), dqkv.data_ptr(), dqkv.stride(0),
                                   B, T, H, H, hd, 0, seed, p, mask.data_ptr(),
                                   bp.data_ptr() if bp is not None else None, bp.stride(0) if bp is not None else 0,
                                   ws.data_ptr(), ws.numel() * 4, st) == 0

        def msk():
            assert lib.cg_attn_drop_mask(B, T, H, seed, p, mask.data_ptr(), st) == 0

        res = {"lib": str(path)}
        for name, fn in (("mask", msk), ("fwd", fwd), ("bwd_bias", lambda: bwd(bpart)), ("bwd", lambda: bwd(None))):
            for _ in range(10):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            n = 20
            e0.record()
            for _ in range(n):
                fn()
            e1.record()
            torch.cuda.synchronize()
            res[name + "_us"] = round(e0.elapsed_time(e1) * 1000 / n, 1)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
