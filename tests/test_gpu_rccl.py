"""RCCL (the ROCm `nccl` backend) on the real engine, world size 1 (marker ``gpu``).

The box has one MI355X, and RCCL wants a GPU per rank, so the multi-rank exchange is covered by
the gloo tests (tests/test_gpu_ddp.py, tests/test_gpu_trainer_ddp.py) and the driver's 8-GPU run.
This smoke exercises what those cannot: RCCL's initialisation on the device and the bucketed
async all-reduces of DataParallelStep issued on RCCL's stream while the native backward keeps
running (``always_reduce`` issues them at world 1, where each is an identity).  The gradients
and the AdamW result must equal a step without any collective, and every bucket
must have been reduced (the averaging contract of loop.py:145-150 at world 1).
"""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        from codonlm_amd import TinyGPT
        from codonlm_amd.optim import FusedAdamW
        from codonlm_amd.training.ddp import DataParallelStep, bucket_ranges
        rng = np.random.default_rng(21)
        t = torch.from_numpy(rng.integers(4, 68, size=(4, 257)))
        t[:, 100] = 3
        x, y = t[:, :-1].contiguous().to(dev), t[:, 1:].contiguous().to(dev)
        res = {"backend": dist.get_backend()}
        for name, always in (("rccl", True), ("none", False)):
            torch.manual_seed(7)
            m = TinyGPT(68, 256, n_layer=4, n_head=4, n_embd=128, dropout=0.1, label_smoothing=0.05,
                        compute_dtype="bf16", device=dev)
            m.train()
            st = DataParallelStep(m, FusedAdamW(m, lr=1e-3), always_reduce=always)
            _, handles = st.microbatch(x, y, seed=3, accumulate=False, sync=True)
            for h in handles:
                h.wait()
            g = m.flat_grads().detach().cpu().clone()
            st.opt.step(grad_scale=1.0)
            torch.cuda.synchronize()
            res[name] = (g, m.flat_parameters().detach().cpu().clone(), len(handles))
        res["buckets"] = sum(1 for b, e in bucket_ranges(m).values() if e > b)
        out[0] = res
    finally:
        dist.destroy_process_group()


def test_rccl_world1_data_parallel_step():
    out = mp.Manager().dict()
    mp.spawn(_worker, args=(_free_port(), out), nprocs=1, join=True)
    r = out[0]
    assert r["backend"] == "nccl"
    g1, p1, n1 = r["rccl"]
    g0, p0, n0 = r["none"]
    assert n0 == 0 and n1 == r["buckets"] >= 3, (n1, r["buckets"])
    assert float(g0.abs().sum()) > 0
    # (the same kernels on the same inputs; a tolerance in case a reduction order differs)
    assert float((g1 - g0).abs().max()) <= 1e-6 * float(g0.abs().max()), "the all-reduce changed the gradients"
    assert float((p1 - p0).abs().max()) <= 1e-6 * float(p0.abs().max())
