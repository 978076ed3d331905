"""Trainer on the MI355X: device-resident batches and the reference loop's counters.

* gather kernels vs numpy and the reference loaders' batch order (golden data_order.npz);
* tests/test_nonfinite_accumulation.py:76-135 of the reference re-expressed: a NaN loss on the
  2nd train microbatch aborts the group, the checkpoint carries the reference counters, and
  resume replays to step 2 / 12 consumed tokens (model widened to d=64: the engine's head
  dims; the counters do not depend on width);
* an end-to-end run with the aux heads writes the reference's run files.
"""
import csv
import json
from types import SimpleNamespace

import numpy as np
import pytest
import torch
import yaml

from conftest import load_golden

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("dtype", [np.int32, np.uint8, np.int16, np.int64])
def test_gather_windows_and_sequences(tmp_path, dtype):
    from codonlm_amd.data_loading import DeviceCodonDataset
    rng = np.random.default_rng(1)
    X = rng.integers(0, 69, size=(50, 33)).astype(dtype)
    Y = rng.integers(0, 69, size=(50, 33)).astype(dtype)
    np.savez(tmp_path / "f.npz", X=X, Y=Y)
    ds = DeviceCodonDataset([tmp_path / "f.npz"], DEV)
    rows = np.array([3, 49, 0, 7, 7], dtype=np.int64)
    x, y = ds.gather(torch.from_numpy(rows).to(DEV), rows)
    assert np.array_equal(x.cpu().numpy(), X[rows].astype(np.int64))
    assert np.array_equal(y.cpu().numpy(), Y[rows].astype(np.int64))
    lens = rng.integers(2, 40, size=30)
    flat = rng.integers(1, 69, size=int(lens.sum())).astype(dtype)
    # two files: offsets restart per file in the reference; one global store here
    np.savez(tmp_path / "d1.npz", X=flat[: lens[:10].sum()], lengths=lens[:10])
    np.savez(tmp_path / "d2.npz", X=flat[lens[:10].sum():], lengths=lens[10:])
    dd = DeviceCodonDataset([tmp_path / "d1.npz", tmp_path / "d2.npz"], DEV)
    starts = np.concatenate([[0], np.cumsum(lens[:-1])])
    rows = np.array([0, 9, 10, 29, 15], dtype=np.int64)
    x, y = dd.gather(torch.from_numpy(rows).to(DEV), rows)
    Tout = int(lens[rows].max()) - 1
    for i, r in enumerate(rows):
        s = flat[starts[r]: starts[r] + lens[r]].astype(np.int64)
        ex = np.zeros(Tout, np.int64)
        ey = np.zeros(Tout, np.int64)
        ex[: len(s) - 1], ey[: len(s) - 1] = s[:-1], s[1:]
        assert np.array_equal(x[i].cpu().numpy(), ex) and np.array_equal(y[i].cpu().numpy(), ey)


@pytest.mark.parametrize("dtype", [np.int32, np.uint8, np.int16])
def test_npy_mmap_sidecars(tmp_path, dtype, monkeypatch):
    """use_mmap (MmapPackedDataset, data_loading.py:132-200): uncompressed <stem>_X / _Y /
    _lengths .npy sidecars are memory-mapped and streamed to HBM (here in 1000-element pieces, so
    chunk seams fall inside rows); the gathered batches equal the NPZ path's.  A path without
    sidecars falls back to the NPZ, as the reference does."""
    from codonlm_amd import data_loading as DL
    monkeypatch.setattr(DL, "_CHUNK", 1000)
    rng = np.random.default_rng(2)
    X = rng.integers(0, 69, size=(70, 65)).astype(dtype)
    Y = rng.integers(0, 69, size=(70, 65)).astype(dtype)
    np.savez_compressed(tmp_path / "f.npz", X=X, Y=Y)
    np.save(tmp_path / "f_X.npy", X)
    np.save(tmp_path / "f_Y.npy", Y)
    rows = np.array([3, 69, 0, 7, 7, 40], dtype=np.int64)
    rd = torch.from_numpy(rows).to(DEV)
    a = DL.DeviceCodonDataset([tmp_path / "f.npz"], DEV, use_mmap=True)
    b = DL.DeviceCodonDataset([tmp_path / "f.npz"], DEV, use_mmap=False)
    assert a.storage_mode == "npy_mmap" and b.storage_mode == "npz_memory" and len(a) == len(b) == 70
    for u, v in zip(a.gather(rd, rows), b.gather(rd, rows)):
        assert torch.equal(u, v)
    assert np.array_equal(a.gather(rd, rows)[0].cpu().numpy(), X[rows].astype(np.int64))
    # dynamic: flat X + lengths over two shards
    lens = rng.integers(2, 80, size=40)
    flat = rng.integers(1, 69, size=int(lens.sum())).astype(dtype)
    cut = int(lens[:15].sum())
    for name, fx, ln in (("d1", flat[:cut], lens[:15]), ("d2", flat[cut:], lens[15:])):
        np.savez(tmp_path / f"{name}.npz", X=fx, lengths=ln)
        np.save(tmp_path / f"{name}_X.npy", fx)
        np.save(tmp_path / f"{name}_lengths.npy", ln)
    paths = [tmp_path / "d1.npz", tmp_path / "d2.npz"]
    a = DL.DeviceCodonDataset(paths, DEV, use_mmap=True)
    b = DL.DeviceCodonDataset(paths, DEV)
    assert a.storage_mode == "npy_mmap" and a.is_dynamic and np.array_equal(a.seq_lengths, b.seq_lengths)
    rows = np.array([0, 14, 15, 39, 22], dtype=np.int64)
    rd = torch.from_numpy(rows).to(DEV)
    for u, v in zip(a.gather(rd, rows), b.gather(rd, rows)):
        assert torch.equal(u, v)
    # no sidecar for one shard -> the NPZ path for all (the reference's fallback)
    (tmp_path / "d2_X.npy").unlink()
    c = DL.DeviceCodonDataset(paths, DEV, use_mmap=True)
    assert c.storage_mode == "npz_memory"


def test_device_loader_matches_reference_order(tmp_path):
    from codonlm_amd.data_loading import DeviceBatchLoader, DeviceCodonDataset
    _, g = load_golden("data_order")
    X = np.arange(23 * 5, dtype=np.int32).reshape(23, 5) % 60 + 4
    X[:, 0] = np.arange(23) + 4
    np.savez(tmp_path / "fixed.npz", X=X, Y=(X + 1).astype(np.int32))
    ds = DeviceCodonDataset([tmp_path / "fixed.npz"], DEV)
    got = torch.cat([xb for xb, _ in DeviceBatchLoader(ds, 4, shuffle=True, seed=11)]).cpu().numpy()
    assert np.array_equal(got, g["fixed_seed11_x"])
    np.savez(tmp_path / "dyn.npz", X=g["dyn_flat"], lengths=g["dyn_lengths"])
    dd = DeviceCodonDataset([tmp_path / "dyn.npz"], DEV)
    batches = list(DeviceBatchLoader(dd, 3, shuffle=True, seed=9, bucket_batching=True, n_buckets=4))
    assert len(batches) == int(g["dyn_bucket_batches"])
    for i, (xb, yb) in enumerate(batches):
        assert np.array_equal(xb.cpu().numpy(), g[f"dyn_bucket_x_{i}"])
        assert np.array_equal(yb.cpu().numpy(), g[f"dyn_bucket_y_{i}"])
    # rank sharding: every rank gets floor(n/world) batches, interleaved in the global order
    parts = [list(DeviceBatchLoader(ds, 4, shuffle=True, seed=11, rank=r, world=2)) for r in range(2)]
    assert len(parts[0]) == len(parts[1]) == 3
    inter = torch.cat([torch.cat([parts[0][j][0], parts[1][j][0]]) for j in range(3)]).cpu().numpy()
    assert np.array_equal(inter, g["fixed_seed11_x"])


def _config(tmp_path, **over):
    cfg = {"vocab_size": 69, "block_size": 4, "n_layer": 1, "n_head": 1, "n_embd": 64, "dropout": 0.0,
           "batch_size": 1, "grad_accum_steps": 2, "max_nonfinite_accumulation_groups": 0, "lr": 0.001,
           "min_lr": 0.0001, "weight_decay": 0.0, "warmup_steps": 0, "epochs": 1, "optimizer": "adamw",
           "amp": False, "use_checkpoint": False, "scheduler": "cosine", "early_stop_patience": 2,
           "seed": 42, "num_workers": 0, "compute_dtype": "fp32"}
    cfg.update(over)
    return cfg


def _write_inputs(tmp_path, config, x_train, y_train, x_val, y_val, V=69):
    itos_path = tmp_path / "itos.txt"
    itos_path.write_text("\n".join(f"token_{i}" for i in range(V)) + "\n")
    config["itos_path"] = str(itos_path)
    config_path = tmp_path / "config.yaml"
    config_path.write_text(yaml.safe_dump(config))
    paths = {}
    for name, x, y in (("train", x_train, y_train), ("val", x_val, y_val), ("test", x_val, y_val)):
        p = tmp_path / f"{name}.npz"
        np.savez_compressed(p, X=x, Y=y)
        paths[name] = p
    return config_path, paths


def _args(config_path, paths, *, run_id, resume=None):
    return SimpleNamespace(config=str(config_path), run_id=run_id, resume=resume, transfer_from=None,
                           train_npz=[str(paths["train"])], val_npz=[str(paths["val"])],
                           test_npz=[str(paths["test"])])


def test_nonfinite_abort_checkpoint_and_resume_preserve_step_counters(tmp_path, monkeypatch):
    from codonlm_amd.model_tiny_gpt import TinyGPT
    from codonlm_amd.training.loop import NonfiniteGroupLimitError, run_training
    monkeypatch.chdir(tmp_path)
    config = _config(tmp_path)
    config_path, paths = _write_inputs(tmp_path, config, np.ones((5, 4), np.int32), np.full((5, 4), 2, np.int32),
                                       np.ones((2, 4), np.int32), np.full((2, 4), 2, np.int32))
    original_forward = TinyGPT.forward
    train_calls = 0

    def fail_second_train_microbatch(self, *args, **kwargs):
        nonlocal train_calls
        result = original_forward(self, *args, **kwargs)
        if self.training:
            train_calls += 1
            if train_calls == 2:
                logits, loss = result
                return logits, loss * torch.tensor(float("nan"), device=loss.device)
        return result

    monkeypatch.setattr(TinyGPT, "forward", fail_second_train_microbatch)
    args = _args(config_path, paths, run_id="nonfinite-resume")
    with pytest.raises(NonfiniteGroupLimitError):
        run_training(dict(config), args)
    ckpt_path = tmp_path / "runs/nonfinite-resume/checkpoints/last.pt"
    ck = torch.load(ckpt_path, map_location="cpu", weights_only=True)
    assert ck["step"] == 0
    assert ck["consumed_train_tokens"] == 0
    assert ck["scheduler"]["last_epoch"] == 0
    assert ck["epoch_microbatch_idx"] == 2
    assert ck["epoch_train_metrics"]["microbatches"] == 0
    assert ck["accumulation_health"] == {"active_microbatches": 0, "nonfinite_microbatches": 1,
                                         "aborted_groups": 1, "discarded_finite_microbatches": 1}
    assert ck["cfg"]["vocabulary"]["size"] == 69
    assert ck["cfg"]["vocabulary"]["legacy_adaptation"] is False
    assert (tmp_path / "runs/nonfinite-resume/itos.txt").exists()
    assert (tmp_path / "runs/nonfinite-resume/vocabulary.json").exists()
    meta = json.loads((tmp_path / "runs/nonfinite-resume/checkpoints/meta.json").read_text())
    assert meta["status"] == "failed" and meta["error_type"] == "NonfiniteGroupLimitError"

    monkeypatch.setattr(TinyGPT, "forward", original_forward)
    run_training(dict(config), _args(config_path, paths, run_id="nonfinite-resume", resume=str(ckpt_path)))
    resumed = torch.load(ckpt_path, map_location="cpu", weights_only=True)
    assert resumed["step"] == 2
    assert resumed["consumed_train_tokens"] == 12
    assert resumed["scheduler"]["last_epoch"] == 2
    assert resumed["epoch_microbatch_idx"] == 0
    assert resumed["epoch_train_metrics"]["microbatches"] == 3
    assert resumed["accumulation_health"]["aborted_groups"] == 1
    assert resumed["accumulation_health"]["discarded_finite_microbatches"] == 1
    assert resumed["optimizer"]["flat_state"]["step"] == 2


def test_end_to_end_run_with_aux_heads(tmp_path, monkeypatch):
    from codonlm_amd.training.loop import run_training
    monkeypatch.chdir(tmp_path)
    rng = np.random.default_rng(0)
    T = 32
    seq = rng.integers(4, 68, size=(24, T + 1)).astype(np.int32)
    seq[:, 0] = 1
    seq[:, 15] = 2
    seq[:, 16] = 3
    seq[:, 17] = 1
    seq[-1, -5:] = 0
    config = _config(tmp_path, vocab_size=68, block_size=T, n_layer=2, n_head=1, batch_size=4, grad_accum_steps=2,
                     epochs=2, multi_offset_loss_enabled=True, multi_offset_targets=[2, 4],
                     termination_loss_enabled=True, termination_class_weights=[1.0, 2.0, 1.5, 1.0, 0.5],
                     eos_loss_weight=3.0, label_smoothing=0.05, compute_dtype="bf16", lr=3e-3, warmup_steps=2,
                     save_epochs=True)
    config_path, paths = _write_inputs(tmp_path, config, seq[:20, :-1], seq[:20, 1:], seq[20:, :-1], seq[20:, 1:],
                                       V=68)
    run_training(dict(config), _args(config_path, paths, run_id="aux-run"))
    run = tmp_path / "runs/aux-run"
    rows = list(csv.reader((run / "scores/curves.csv").open()))
    assert rows[0] == ["step", "train_loss", "val_loss", "train_next_loss", "val_next_loss", "perplexity", "lr",
                       "train_offset_2", "val_offset_2", "train_offset_4", "val_offset_4", "train_term_loss",
                       "val_term_loss"]
    assert len(rows) == 3 and all(np.isfinite(float(v)) for v in rows[2][1:])
    metrics = json.loads((run / "scores/metrics.json").read_text())
    assert metrics["status"] == "completed" and metrics["last_epoch"] == 2
    for name in ("last.pt", "best.pt", "epoch_1.pt", "epoch_2.pt"):
        assert (run / "checkpoints" / name).exists(), name
    ck = torch.load(run / "checkpoints/last.pt", map_location="cpu", weights_only=True)
    assert ck["step"] == 6  # 5 microbatches/epoch, gacc 2 -> 3 commits per epoch
    assert ck["consumed_train_tokens"] == 20 * T * 2  # no PAD in the train split
    assert set(ck["model"]).issuperset({"termination_head.weight", "offset_projs.2.0.weight", "tok_emb.weight"})
    assert ck["epoch"] == 2 and ck["epoch_microbatch_idx"] == 0
    # the state dict loads strictly into a fresh model (resume uses strict load, loop.py:882)
    from codonlm_amd.training.loop import build_model
    m = build_model(dict(ck["cfg"]), DEV)
    m.load_state_dict(ck["model"])


def test_transfer_from_cfg_remaps_vocabulary_and_runs(tmp_path, monkeypatch):
    """stage2.6_large_scaling-style warm start (configs/stage2.6_large_scaling.yaml:16): the cfg
    key transfer_from loads a previous run's checkpoint into a deeper model with a different
    vocabulary through the reference's row remapping (training/checkpoint.py:16-85,
    loop.py:266,824-877); device: mps (the primary contracts' pin) runs on the MI355X."""
    from codonlm_amd.training.loop import run_training
    monkeypatch.chdir(tmp_path)
    rng = np.random.default_rng(2)
    T = 32
    seq = rng.integers(4, 68, size=(12, T + 1)).astype(np.int32)
    src_cfg = _config(tmp_path, vocab_size=69, block_size=T, n_layer=1, n_head=1, batch_size=4, grad_accum_steps=1,
                      epochs=1, compute_dtype="bf16")
    config_path, paths = _write_inputs(tmp_path, src_cfg, seq[:8, :-1], seq[:8, 1:], seq[8:, :-1], seq[8:, 1:], V=69)
    run_training(dict(src_cfg), _args(config_path, paths, run_id="src-run"))
    src_ck = tmp_path / "runs/src-run/checkpoints/last.pt"
    src = torch.load(src_ck, map_location="cpu", weights_only=True)["model"]
    # target: 68 tokens with the source's token_5 / token_6 swapped and token_7 renamed, 2 layers
    tgt_dir = tmp_path / "tgt"
    tgt_dir.mkdir()
    itos = [f"token_{i}" for i in range(68)]
    itos[5], itos[6], itos[7] = "token_6", "token_5", "novel"
    (tgt_dir / "itos.txt").write_text("\n".join(itos) + "\n")
    tgt_cfg = _config(tgt_dir, vocab_size=68, block_size=T, n_layer=2, n_head=1, batch_size=4, grad_accum_steps=1,
                      epochs=1, compute_dtype="bf16", lr=0.0, min_lr=0.0, device="mps",
                      transfer_from=str(src_ck), itos_path=str(tgt_dir / "itos.txt"))
    tgt_cfg_path = tgt_dir / "config.yaml"
    tgt_cfg_path.write_text(yaml.safe_dump(tgt_cfg))
    run_training(dict(tgt_cfg), _args(tgt_cfg_path, paths, run_id="tgt-run"))
    ck = torch.load(tmp_path / "runs/tgt-run/checkpoints/last.pt", map_location="cpu", weights_only=True)
    emb, semb = ck["model"]["tok_emb.weight"], src["tok_emb.weight"]
    # lr 0: the trained weights are exactly the transferred ones
    assert torch.equal(emb[5], semb[6]) and torch.equal(emb[6], semb[5]) and torch.equal(emb[20], semb[20])
    assert not torch.equal(emb[7], semb[7])
    assert torch.equal(ck["model"]["blocks.0.attn.query.weight"], src["blocks.0.attn.query.weight"])
    voc = ck["cfg"]["vocabulary"]
    assert voc["legacy_adaptation"] is True and voc["transfer"]["source_embedding_rows"] == 69
    assert "tok_emb.weight:67" in voc["transfer"]["loaded_rows"]
    assert json.loads((tmp_path / "runs/tgt-run/vocabulary.json").read_text())["transfer"]["checkpoint"] == str(src_ck)
    assert ck["cfg"]["device_contract"] == "mps" and ck["cfg"]["device"].startswith("cuda")
    assert "transfer_from" not in ck["cfg"]  # consumed like the reference's cfg.pop


def test_bf16_training_on_dynamic_length_batches(tmp_path, monkeypatch):
    """The dynamic-length loader (flat X + lengths, data_loading.py:380-393) pads each batch only
    to its own longest sequence, so B*T is arbitrary; the bf16 engine (the trainer's default
    compute dtype) trains on such batches -- the grouped weight-gradient launch reduces over any
    token count (a zero-filled ragged last k-step), with dropout on and bucketed batches."""
    from codonlm_amd.engine import Engine
    from codonlm_amd.training.loop import run_training
    monkeypatch.chdir(tmp_path)
    rng = np.random.default_rng(7)
    T = 128
    lens = rng.integers(20, T + 1, size=40)
    flat = rng.integers(4, 68, size=int(lens.sum())).astype(np.int32)
    for name, sl in (("train", slice(0, 30)), ("val", slice(30, 40)), ("test", slice(30, 40))):
        s = np.concatenate([[0], np.cumsum(lens)])
        parts = [flat[s[i]:s[i + 1]] for i in range(len(lens))][sl]
        np.savez(tmp_path / f"{name}.npz", X=np.concatenate(parts), lengths=lens[sl])
    config = _config(tmp_path, vocab_size=68, block_size=T, n_layer=3, n_head=2, n_embd=128, batch_size=3,
                     grad_accum_steps=2, epochs=2, dropout=0.1, label_smoothing=0.05, compute_dtype="bf16",
                     lr=3e-3, warmup_steps=1, bucket_batching=True, n_buckets=3)
    itos = tmp_path / "itos.txt"
    itos.write_text("\n".join(f"token_{i}" for i in range(68)) + "\n")
    config["itos_path"] = str(itos)
    cp = tmp_path / "config.yaml"
    cp.write_text(yaml.safe_dump(config))
    shapes = []
    orig = Engine.forward

    def record(self, idx, targets, **kw):
        shapes.append(tuple(idx.shape))
        return orig(self, idx, targets, **kw)

    monkeypatch.setattr(Engine, "forward", record)
    paths = {k: tmp_path / f"{k}.npz" for k in ("train", "val", "test")}
    run_training(dict(config), _args(cp, paths, run_id="dyn-bf16"))
    ragged = [s for s in shapes if (s[0] * s[1]) % 64]
    assert len(ragged) >= len(shapes) // 2, shapes
    rows = list(csv.reader((tmp_path / "runs/dyn-bf16/scores/curves.csv").open()))
    assert len(rows) == 3 and all(np.isfinite(float(v)) for v in rows[2][1:3])
    metrics = json.loads((tmp_path / "runs/dyn-bf16/scores/metrics.json").read_text())
    assert metrics["status"] == "completed"
    ck = torch.load(tmp_path / "runs/dyn-bf16/checkpoints/last.pt", map_location="cpu", weights_only=True)
    # every train target that is not PAD, both epochs (the reference's consumed_train_tokens)
    assert ck["consumed_train_tokens"] == 2 * int((lens[:30] - 1).sum())
    assert ck["step"] >= 10 and ck["epoch"] == 2
    assert all(torch.isfinite(v).all() for k, v in ck["model"].items() if v.is_floating_point())


def test_oom_safeguard_checkpoints_and_downscales_config(tmp_path, monkeypatch):
    """loop.py:1501-1549: an allocation failure inside the loop saves last.pt with
    checkpoint_reason "oom", halves batch_size / doubles grad_accum_steps in the YAML, re-raises."""
    from codonlm_amd.engine import Engine
    from codonlm_amd.training.loop import run_training
    monkeypatch.chdir(tmp_path)
    rng = np.random.default_rng(4)
    seq = rng.integers(4, 68, size=(16, 33)).astype(np.int32)
    config = _config(tmp_path, vocab_size=68, block_size=32, batch_size=4, grad_accum_steps=2, epochs=1,
                     compute_dtype="bf16")
    config_path, paths = _write_inputs(tmp_path, config, seq[:12, :-1], seq[:12, 1:], seq[12:, :-1], seq[12:, 1:],
                                       V=68)
    orig = Engine._ensure_workspace
    calls = {"n": 0}

    def failing(self, B, T):
        calls["n"] += 1
        if calls["n"] == 3:
            raise torch.cuda.OutOfMemoryError("HIP out of memory. Tried to allocate 288.00 GiB")
        return orig(self, B, T)

    monkeypatch.setattr(Engine, "_ensure_workspace", failing)
    with pytest.raises(torch.cuda.OutOfMemoryError):
        run_training(dict(config), _args(config_path, paths, run_id="oom-run"))
    ck = torch.load(tmp_path / "runs/oom-run/checkpoints/last.pt", map_location="cpu", weights_only=True)
    assert ck["checkpoint_reason"] == "oom"
    assert ck["step"] == 1  # the first group of 2 committed before the failing 3rd microbatch
    new = yaml.safe_load(config_path.read_text())
    assert new["batch_size"] == 2 and new["grad_accum_steps"] == 4
