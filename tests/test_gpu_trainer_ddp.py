"""`run_training` itself at world size 2 (marker ``gpu``; both ranks share the box's MI355X and
talk over gloo -- RCCL needs a GPU per rank, which the driver's multi-GPU run covers).

The trainer's world > 1 path (training/loop.py: the bucket hook handed to the group-completing
microbatch's backward, drain() on abort and at group end, the collective abort / wall-time
decisions of training/stepper.py, token and val sums over the control group, val batches
sharded without a drop) must keep every rank in the same collective sequence -- a mismatch
hangs the job -- and must reproduce the single-process semantics of the reference loop
(src/codonlm/training/loop.py:1054-1261):

* a clean run: both ranks end with identical weights, equal (fp32 engine, dropout 0) to ONE
  process training the same global batch order with grad_accum_steps doubled -- the DP group of
  g microbatches per rank is the reference's group of 2g microbatches, averaged over 2g; an odd
  number of batches per rank leaves a partial last group each epoch, and the val split has an
  uneven number of batches per rank;
* a nonfinite loss on rank 1's group-completing microbatch aborts that group on BOTH ranks
  (identical AccumulationHealth counters, no optimizer step, no hang);
* the wall-time limit stops both ranks at the same microbatch (status "stopped").
"""
import json
import os
import socket
from types import SimpleNamespace

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import yaml

pytestmark = pytest.mark.gpu

T = 32


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup(root, **over):
    rng = np.random.default_rng(3)
    seq = rng.integers(4, 68, size=(26, T + 1)).astype(np.int32)
    seq[:, 10] = 3
    cfg = {"vocab_size": 68, "block_size": T, "n_layer": 2, "n_head": 2, "n_embd": 64, "dropout": 0.0,
           "batch_size": 2, "grad_accum_steps": 2, "max_nonfinite_accumulation_groups": 3, "lr": 3e-3,
           "min_lr": 1e-4, "weight_decay": 0.05, "warmup_steps": 1, "epochs": 2, "optimizer": "adamw",
           "scheduler": "cosine", "early_stop_patience": 5, "seed": 42, "compute_dtype": "fp32",
           "label_smoothing": 0.05}
    cfg.update(over)
    itos = root / "itos.txt"
    itos.write_text("\n".join(f"token_{i}" for i in range(68)) + "\n")
    cfg["itos_path"] = str(itos)
    # 20 train rows -> 10 batches of 2 -> 5 per rank: groups of 2, 2 and a partial 1 per epoch;
    # 6 val rows -> 3 batches -> 2 on rank 0, 1 on rank 1
    np.savez(root / "train.npz", X=seq[:20, :-1], Y=seq[:20, 1:])
    np.savez(root / "val.npz", X=seq[20:, :-1], Y=seq[20:, 1:])
    cp = root / "config.yaml"
    cp.write_text(yaml.safe_dump(cfg))
    return cfg, cp


def _args(root, cp, run_id):
    return SimpleNamespace(config=str(cp), run_id=run_id, resume=None, transfer_from=None,
                           train_npz=[str(root / "train.npz")], val_npz=[str(root / "val.npz")],
                           test_npz=[str(root / "val.npz")])


def _worker(rank, world, port, root, cfg, cp, run_id, mode, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LOCAL_RANK=str(rank))
    os.chdir(root)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from codonlm_amd.model_tiny_gpt import TinyGPT
        from codonlm_amd.training import loop
        res = {}
        if mode == "nan":
            orig = TinyGPT.forward
            calls = {"n": 0}

            def fwd(self, *a, **k):
                r = orig(self, *a, **k)
                if self.training and rank == 1:
                    calls["n"] += 1
                    if calls["n"] == 2:  # rank 1's 2nd microbatch completes the first group
                        return (r[0], r[1] * torch.tensor(float("nan"), device=r[1].device)) + tuple(r[2:])
                return r
            TinyGPT.forward = fwd
        captured = {}
        orig_finish = loop._finish

        def finish(is_main, ckpt_dir, scores_dir, run_id_, t_wall0, st, health, model, history, status):
            captured.update(step=st.step, consumed=st.consumed, health=health.state_dict(), status=status,
                            flat=model.flat_parameters().detach().cpu().clone(),
                            named={k: v.detach().cpu().clone() for k, v in model.named_parameters()})
            return orig_finish(is_main, ckpt_dir, scores_dir, run_id_, t_wall0, st, health, model, history, status)
        loop._finish = finish
        loop.run_training(dict(cfg), _args(root, cp, run_id))
        res.update(captured)
        dist.barrier()
        out[rank] = res
    finally:
        dist.destroy_process_group()


def _spawn(args, timeout=240):
    """Two ranks; a rank that hangs (mismatched collectives) fails the test instead of the session."""
    ctx = mp.start_processes(_worker, args=args, nprocs=2, join=False, start_method="spawn")
    waited = 0
    while not ctx.join(timeout=5):
        waited += 5
        if waited >= timeout:
            for p in ctx.processes:
                if p.is_alive():
                    p.kill()
            pytest.fail("world-2 run_training did not finish: ranks out of collective step")


def _run(tmp_path, mode, **over):
    cfg, cp = _setup(tmp_path, **over)
    out = mp.Manager().dict()
    _spawn((2, _free_port(), tmp_path, cfg, cp, f"ddp-{mode}", mode, out))
    return cfg, cp, dict(out)


def test_run_training_world2_matches_single_process(tmp_path, monkeypatch):
    cfg, cp, out = _run(tmp_path, "clean")
    r0, r1 = out[0], out[1]
    assert r0["status"] == r1["status"] == "completed"
    assert r0["step"] == r1["step"] == 6  # 3 commits per rank per epoch (2 + 2 + partial 1), 2 epochs
    assert r0["health"] == r1["health"]
    assert r0["consumed"] == r1["consumed"] == 2 * 10 * 2 * T  # tokens summed over the ranks
    assert torch.equal(r0["flat"], r1["flat"]), "ranks diverged"
    # ONE process over the same global batch order with grad_accum_steps 4: its groups are the
    # union of the ranks' groups (rank r takes global batches r, r+2, ...), the partial last group
    # included (2 microbatches averaged over 2 in both)
    import codonlm_amd.training.loop as loop_mod
    monkeypatch.chdir(tmp_path)
    single = dict(cfg, grad_accum_steps=4)
    cp1 = tmp_path / "single.yaml"
    cp1.write_text(yaml.safe_dump(single))
    got = {}
    orig = loop_mod._finish

    def finish(is_main, ckpt_dir, scores_dir, run_id_, t_wall0, st, health, model, history, status):
        got.update(step=st.step, consumed=st.consumed,
                   named={k: v.detach().cpu().clone() for k, v in model.named_parameters()})
        return orig(is_main, ckpt_dir, scores_dir, run_id_, t_wall0, st, health, model, history, status)
    monkeypatch.setattr(loop_mod, "_finish", finish)
    loop_mod.run_training(dict(single), _args(tmp_path, cp1, "single"))
    assert got["step"] == 6 and got["consumed"] == r0["consumed"]
    # attn.key.bias has an exactly-zero gradient in exact arithmetic (softmax shift invariance):
    # its gradient is rounding noise, which AdamW's normalisation turns into +-lr steps whose sign
    # depends on the summation order -- those tensors are compared to lr * steps only
    for k, ref in got["named"].items():
        err = float((r0["named"][k] - ref).abs().max())
        bound = 2 * 6 * 3e-3 if k.endswith("attn.key.bias") else 1e-4 * max(1.0, float(ref.abs().max()))
        assert err <= bound, (k, err, bound)
    # the val loss is the same mean over the 3 val batches (2 on rank 0 + 1 on rank 1)
    import csv
    dp_rows = list(csv.reader((tmp_path / "runs/ddp-clean/scores/curves.csv").open()))
    sp_rows = list(csv.reader((tmp_path / "runs/single/scores/curves.csv").open()))
    assert abs(float(dp_rows[-1][2]) - float(sp_rows[-1][2])) <= 2e-3


def test_run_training_world2_collective_abort(tmp_path):
    _, _, out = _run(tmp_path, "nan")
    r0, r1 = out[0], out[1]
    assert r0["health"] == r1["health"]
    assert r0["health"]["aborted_groups"] == 1 and r0["health"]["nonfinite_microbatches"] == 1
    assert r0["health"]["discarded_finite_microbatches"] == 1
    assert r0["step"] == r1["step"] == 5  # the aborted group's commit is lost on both ranks
    assert torch.equal(r0["flat"], r1["flat"])


def test_run_training_world2_wall_time_stop(tmp_path):
    _, _, out = _run(tmp_path, "wall", max_time_minutes=1e-6)
    r0, r1 = out[0], out[1]
    assert r0["status"] == r1["status"] == "stopped"
    assert r0["step"] == r1["step"]
    assert torch.equal(r0["flat"], r1["flat"])
    meta = json.loads((tmp_path / "runs/ddp-wall/checkpoints/meta.json").read_text())
    assert meta["status"] == "stopped"
