"""Codon-LM training loop on the MI355X engine (mirrors src/codonlm/training/loop.py run_training).

Same config keys, defaults, counters, checkpoint payload and files as the reference trainer
so runs, resumes and downstream tools interchange:

* microbatch loop (loop.py:1016-1285): loss is NOT divided by grad_accum_steps; grads are
  summed and averaged over the actual group size at commit (``_average_accumulated_gradients``
  :145-150 -- folded into the fused AdamW launch as ``grad_scale``), including the partial
  last group of an epoch; a nonfinite microbatch aborts the group (AccumulationHealth
  :90-142) and ``max_nonfinite_accumulation_groups`` bounds the aborts (NonfiniteGroupLimitError);
* optimizer (:681-731): the reference's two param groups (fast group = offset_projs /
  termination_head with lr_embedding and wd 0; backbone incl. embeddings with lr / weight_decay);
* scheduler (:733-792): cosine-with-warmup LambdaLR stepped per committed group, or
  ReduceLROnPlateau on the val loss with the manual linear warmup (:1151-1154);
* objectives (:1075-1112): next-codon CE + multi-offset + termination heads (objectives.py);
* per epoch: val pass, curves.csv row, last/best/best_epoch_NNN(/epoch_N) checkpoints written
  atomically with the reference payload keys (:950-1007), early stopping (:1375-1448);
* resume (:879-942) skips already-applied microbatches of the interrupted epoch; wall-time
  limit (:1459-1500); metrics.json / meta.json (:1556-1597).

* warm start (loop.py:266,824-877): ``--transfer_from`` or the cfg key ``transfer_from``
  (ignored on resume) loads a checkpoint with the vocabulary-remapping transfer load
  (training/checkpoint.py) and records the transfer provenance in vocabulary.json;
* corrected primary configs (loop.py:174-195) are validated fail-closed
  (training/primary_contract.py); their pinned ``device: mps`` runs on the MI355X engine.

MI355X-first differences: token stores live in HBM and batches are gathered on the device
(data_loading.py here); fwd+CE+bwd run in the native engine; with torch.distributed
initialised each rank takes every world-th batch, the last microbatch of a group hands the
bucketed RCCL all-reduce to the backward (each block's gradient range is reduced while the
blocks below it are still in backward; 1/world folded into AdamW), the nonfinite-abort and
wall-time decisions are one collective per microbatch over a CPU process group
(training/stepper.py), and the rank is mixed into the dropout seeds.  Per microbatch the
host reads the loss values once, through an event recorded after the forward, so the
backward's kernels keep the GPU busy meanwhile; nothing else synchronises.

Outside the MI355X hot path and rejected with a clear error: shape guidance / biophysics
encoder, replay-termination loss, Adafactor, freeze_backbone, torch.compile (ignored: the
engine is already native), dataset manifests (not enforced).
"""
from __future__ import annotations

import csv
import hashlib
import json
import math
import os
import random
import shutil
import time
from dataclasses import dataclass
from pathlib import Path
from types import SimpleNamespace

import numpy as np
import torch
import torch.distributed as dist

from ..data_loading import DeviceBatchLoader, DeviceCodonDataset
from ..model_tiny_gpt import TinyGPT
from ..optim import FusedAdamW
from . import objectives as obj
from .checkpoint import load_transfer_state_dict, transfer_source_itos
from .ddp import DataParallelStep
from .primary_contract import validate_primary_training_config
from .stepper import GroupController, control_group

RUN_ID_ENV = "RUN_ID"
PAD_ID = 0
# codon_tokenize.py:29-36: specials then the 64 codons in ACGT order
SPECIALS = ["<PAD>", "<BOS_CDS>", "<EOS_CDS>", "<SEP>"]
CODONS = [a + b + c for a in "ACGT" for b in "ACGT" for c in "ACGT"]
VOCAB = SPECIALS + CODONS
STOI = {t: i for i, t in enumerate(VOCAB)}
STOP_CODONS = ("TAA", "TAG", "TGA")


class NonfiniteGroupLimitError(RuntimeError):
    """Raised when aborted accumulation groups exceed the configured tolerance."""


class WallTimeLimitException(Exception):
    pass


def resolve_warmup_steps(cfg: dict, total_steps: int) -> int:
    """loop.py:70-87."""
    if total_steps <= 0:
        raise ValueError("scheduler_total_steps must be positive")
    fraction = cfg.get("warmup_fraction")
    if fraction is None:
        steps = int(cfg.get("warmup_steps", 200))
        if steps < 0:
            raise ValueError("warmup_steps must be non-negative")
        return steps
    if "warmup_steps" in cfg:
        raise ValueError("configure only one of warmup_steps or warmup_fraction")
    fraction = float(fraction)
    if not 0.0 <= fraction < 1.0:
        raise ValueError("warmup_fraction must be in [0, 1)")
    if fraction == 0.0:
        return 0
    return max(1, int(round(total_steps * fraction)))


def normalize_offset_weights(offsets, weights_cfg=None) -> dict:
    """training/config.py:61-74."""
    offsets = [int(o) for o in offsets]
    if not offsets:
        return {}
    if weights_cfg is None:
        return {o: 1.0 / len(offsets) for o in offsets}
    if isinstance(weights_cfg, dict):
        return {o: float(weights_cfg.get(o, weights_cfg.get(str(o), 0.0))) for o in offsets}
    if isinstance(weights_cfg, (list, tuple)):
        if len(weights_cfg) != len(offsets):
            raise ValueError("multi_offset_weights list must match multi_offset_targets length")
        return {o: float(w) for o, w in zip(offsets, weights_cfg)}
    return {o: float(weights_cfg) for o in offsets}


def cosine_lr_lambda(warmup_steps: int, total_steps: int, base_lr: float, min_lr: float):
    """loop.py:773-782."""
    warm = max(1, warmup_steps)
    r = (min_lr / base_lr) if base_lr > 0 else 0.0

    def lr_lambda(step_idx: int) -> float:
        if step_idx < warm:
            return float(step_idx + 1) / warm
        progress = (step_idx - warm) / max(1, total_steps - warm)
        return r + (1 - r) * 0.5 * (1.0 + math.cos(math.pi * progress))
    return lr_lambda


@dataclass
class AccumulationHealth:
    """Checkpointable counters for gradient-accumulation group integrity (loop.py:90-142)."""

    active_microbatches: int = 0
    nonfinite_microbatches: int = 0
    aborted_groups: int = 0
    discarded_finite_microbatches: int = 0

    def record_finite_microbatch(self) -> None:
        self.active_microbatches += 1

    def complete_group(self) -> None:
        if self.active_microbatches <= 0:
            raise ValueError("cannot complete an empty accumulation group")
        self.active_microbatches = 0

    def abort_group(self, optimizer) -> int:
        discarded = self.active_microbatches
        optimizer.zero_grad(set_to_none=True)
        self.nonfinite_microbatches += 1
        self.aborted_groups += 1
        self.discarded_finite_microbatches += discarded
        self.active_microbatches = 0
        return discarded

    def exceeds_limit(self, max_aborted_groups: int) -> bool:
        if max_aborted_groups < 0:
            return False
        return self.aborted_groups > max_aborted_groups

    def state_dict(self) -> dict:
        state = self.metrics_dict()
        state["active_microbatches"] = 0  # grads are not checkpointed
        return state

    def metrics_dict(self) -> dict:
        return {"active_microbatches": self.active_microbatches,
                "nonfinite_microbatches": self.nonfinite_microbatches,
                "aborted_groups": self.aborted_groups,
                "discarded_finite_microbatches": self.discarded_finite_microbatches}

    def load_state_dict(self, state) -> None:
        state = state or {}
        self.active_microbatches = 0
        self.nonfinite_microbatches = int(state.get("nonfinite_microbatches", 0))
        self.aborted_groups = int(state.get("aborted_groups", 0))
        self.discarded_finite_microbatches = int(state.get("discarded_finite_microbatches", 0))


# ------------------------------------------------------------------------------ run files
def capture_rng_state() -> dict:
    """src/training/run_lifecycle.py:84-102 (weights_only-loadable types)."""
    ns = np.random.get_state()
    state = {"python": random.getstate(),
             "numpy": {"bit_generator": ns[0], "state": ns[1].tolist(), "position": int(ns[2]),
                       "has_gauss": int(ns[3]), "cached_gaussian": float(ns[4])},
             "torch_cpu": torch.get_rng_state()}
    if torch.cuda.is_available():
        state["torch_cuda"] = torch.cuda.get_rng_state_all()
    return state


def restore_rng_state(state) -> None:
    if not state:
        return
    random.setstate(state["python"])
    n = state["numpy"]
    np.random.set_state((n["bit_generator"], np.asarray(n["state"], dtype=np.uint32), n["position"],
                         n["has_gauss"], n["cached_gaussian"]))
    torch.set_rng_state(state["torch_cpu"].cpu())
    if "torch_cuda" in state and torch.cuda.is_available():
        torch.cuda.set_rng_state_all([s.cpu() for s in state["torch_cuda"]])


def save_checkpoint_atomic(payload: dict, path: Path) -> None:
    path = Path(path)
    tmp = path.with_name(path.name + f".tmp{os.getpid()}")
    torch.save(payload, tmp)
    os.replace(tmp, path)


def write_meta(run_dir: Path, meta: dict) -> None:
    (Path(run_dir) / "meta.json").write_text(json.dumps(meta, indent=2, sort_keys=True) + "\n")


def _plain(x):
    """cfg -> weights_only-loadable plain types."""
    if isinstance(x, dict):
        return {str(k): _plain(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_plain(v) for v in x]
    if isinstance(x, Path):
        return str(x)
    return x


def _path_list(arg_value, cfg_value, key):
    source = arg_value if arg_value is not None else cfg_value
    if source is None:
        raise ValueError(f"Missing {key} specification (provide in config or CLI)")
    if isinstance(source, (str, os.PathLike)):
        return [str(source)]
    return [str(p) for p in source]


def _read_itos(path):
    if not path:
        return None
    p = Path(path)
    if not p.is_file():
        return None
    return [ln.strip() for ln in p.read_text().splitlines() if ln.strip()]


def _resolve_vocab(cfg: dict):
    itos = _read_itos(cfg.get("itos_path"))
    configured = cfg.get("vocab_size")
    if itos is not None:
        if configured is not None and int(configured) != len(itos):
            raise ValueError(f"vocab_size {configured} does not match itos_path ({len(itos)} tokens)")
        return len(itos), itos
    if configured is not None:
        return int(configured), None
    return len(VOCAB), list(VOCAB)


def _auto_run_id(cfg: dict, config_path) -> str:
    from datetime import date
    tag = "run"
    if config_path:
        stem = Path(config_path).stem
        tag = stem.split("_", 1)[0] if "_" in stem else stem
    return (f"{date.today().strftime('%Y-%m-%d')}_{tag}_{int(cfg.get('n_layer', 0))}L{int(cfg.get('n_head', 0))}H"
            f"_d{int(cfg.get('n_embd', 0))}_e{int(cfg.get('epochs', 0))}")


def configuration_fingerprint(cfg: dict) -> str:
    return hashlib.sha256(json.dumps(_plain(cfg), sort_keys=True, default=str).encode()).hexdigest()


# ------------------------------------------------------------------------------ training
def resolve_device(cfg: dict, local_rank: int = 0) -> torch.device:
    """dev() of loop.py:152-170 on the MI355X path: 'auto' / 'cuda' -> this process's GPU;
    'mps' (pinned by the corrected primary configs) is accepted and runs on the MI355X engine;
    'cpu' is refused (the engine has no CPU path); anything else is a ValueError as in the
    reference."""
    requested = str(cfg.get("device", "auto") or "auto").lower()
    if requested not in {"auto", "cpu", "mps", "cuda"}:
        raise ValueError(f"unsupported device {requested!r}; expected auto, cpu, mps, or cuda")
    if requested == "cpu":
        raise RuntimeError("device=cpu requested, but the codonlm_amd trainer runs only on the MI355X engine "
                           "(train on CPU with the reference trainer)")
    if not torch.cuda.is_available():
        raise RuntimeError(f"requested device={requested} but no MI355X is visible (the codonlm_amd trainer has "
                           "no CPU path)")
    torch.cuda.set_device(local_rank % max(1, torch.cuda.device_count()))
    device = torch.device("cuda", torch.cuda.current_device())
    if requested == "mps":
        cfg["device_contract"] = "mps"
        print(f"[device] device=mps (pinned by the config) -> {device}: the MI355X engine runs the MPS path "
              "(bf16 MFMA compute instead of fp16 autocast; fp32 master weights, loss and optimizer)")
    return device


def build_model(cfg: dict, device) -> TinyGPT:
    """cfg -> TinyGPT kwargs as loop.py:559-579 (plus compute_dtype)."""
    sep_mask_enabled = bool(cfg.get("sep_mask_enabled", True))
    termination_head = bool(cfg.get("termination_loss_enabled", False)) or bool(cfg.get("replay_loss_enabled", False))
    offsets = [int(x) for x in cfg.get("multi_offset_targets", [])] \
        if bool(cfg.get("multi_offset_loss_enabled", False)) else None
    eos_w = cfg.get("eos_loss_weight")
    loss_weights = None
    if eos_w is not None and float(eos_w) != 1.0:
        loss_weights = [1.0] * int(cfg["vocab_size"])
        loss_weights[STOI["<EOS_CDS>"]] = float(eos_w)
        for c in STOP_CODONS:
            if STOI[c] < len(loss_weights):
                loss_weights[STOI[c]] = float(eos_w)
    return TinyGPT(int(cfg["vocab_size"]), int(cfg["block_size"]), n_layer=int(cfg["n_layer"]),
                   n_head=int(cfg["n_head"]), n_embd=int(cfg["n_embd"]), dropout=float(cfg.get("dropout", 0.1)),
                   use_checkpoint=bool(cfg.get("use_checkpoint", cfg.get("grad_checkpointing", False))),
                   label_smoothing=float(cfg.get("label_smoothing", 0.0)),
                   sep_id=(3 if sep_mask_enabled else None), tie_embeddings=bool(cfg.get("tie_embeddings", True)),
                   n_kv_head=int(cfg["n_kv_head"]) if cfg.get("n_kv_head") is not None else None,
                   use_sdpa=bool(cfg.get("use_sdpa", False)), loss_weights=loss_weights,
                   termination_aux=termination_head,
                   termination_n_classes=int(cfg.get("termination_n_classes",
                                                     len(cfg.get("termination_bucket_edges", [0, 3, 10, 30])) + 1)),
                   multi_offset_targets=offsets, use_swiglu=bool(cfg.get("use_swiglu", False)),
                   use_rope=bool(cfg.get("use_rope", False)),
                   compute_dtype=str(cfg.get("compute_dtype", "bf16")), device=device)


def _reject_out_of_scope(cfg: dict) -> None:
    for key, what in (("use_shape_guidance", "shape guidance (biophysics encoder)"),
                      ("replay_loss_enabled", "replay-termination loss"),
                      ("freeze_backbone", "freeze_backbone")):
        if bool(cfg.get(key, False)):
            raise NotImplementedError(f"{what} is outside the MI355X hot path")
    if str(cfg.get("optimizer", "adamw")).lower() != "adamw":
        raise NotImplementedError("only the AdamW optimizer runs on the MI355X path")


def run_training(cfg: dict, args) -> None:
    if cfg.get("primary_training_contract") is not None:  # loop.py:174-195
        contract = validate_primary_training_config(cfg)
        requested = (getattr(args, "run_id", None) or "").strip()
        if requested and requested != contract["run_id"]:
            raise ValueError("--run_id cannot override an immutable primary training config")
        for name in ("train_npz", "val_npz", "test_npz", "transfer_from"):
            if getattr(args, name, None) is not None:
                raise ValueError(f"--{name} cannot override an immutable primary training config")
        print(f"[contract] corrected primary config verified role={contract['role']} "
              f"protocol={contract['protocol']} seed={contract['seed']}")
    _reject_out_of_scope(cfg)
    cfg = dict(cfg)
    resume_path = args.resume or cfg.pop("resume", None)
    resume_path = str(resume_path) if resume_path is not None else None
    for split in ("train", "val", "test"):
        cfg.setdefault(f"{split}_npz", f"data/processed/{split}_bs{cfg['block_size']}.npz")
    train_paths = _path_list(getattr(args, "train_npz", None), cfg.get("train_npz"), "train_npz")
    val_paths = _path_list(getattr(args, "val_npz", None), cfg.get("val_npz"), "val_npz")
    test_paths = _path_list(getattr(args, "test_npz", None), cfg.get("test_npz"), "test_npz")
    cfg["train_npz"], cfg["val_npz"], cfg["test_npz"] = train_paths, val_paths, test_paths
    if "d_head" in cfg and cfg.get("n_head"):
        cfg["n_embd"] = int(cfg["d_head"]) * int(cfg["n_head"])
    vocab_size, itos = _resolve_vocab(cfg)
    cfg["vocab_size"] = vocab_size
    if resume_path and not os.path.isfile(resume_path):
        raise FileNotFoundError(f"Resume checkpoint not found: {resume_path}")
    # loop.py:266 -- CLI or cfg, never on resume (the cfg key is consumed either way)
    cfg_transfer = cfg.pop("transfer_from", None)
    transfer_path = None if resume_path else (getattr(args, "transfer_from", None) or cfg_transfer)
    if transfer_path and not os.path.isfile(transfer_path):
        raise FileNotFoundError(f"Transfer weights not found: {transfer_path}")

    # ---- distributed layout (one process per GPU; RCCL = backend "nccl")
    dist_on = dist.is_available() and dist.is_initialized()
    rank = dist.get_rank() if dist_on else 0
    world = dist.get_world_size() if dist_on else 1
    local = int(os.environ.get("LOCAL_RANK", rank if dist_on else
                               (torch.cuda.current_device() if torch.cuda.is_available() else 0)))
    device = resolve_device(cfg, local)
    cfg["device"] = str(device)
    is_main = rank == 0
    ctrl = control_group(world)

    base_seed = int(cfg.get("seed", 1337))
    # build_codon_lm_datasets(..., use_mmap) (data_loading.py:409): NPY sidecars memory-mapped
    use_mmap = bool(cfg.get("use_mmap", False))
    train_ds = DeviceCodonDataset(train_paths, device, use_mmap=use_mmap)
    val_ds = DeviceCodonDataset(val_paths, device, use_mmap=use_mmap)
    batch_size = int(cfg["batch_size"])

    def train_loader_for(epoch_idx: int) -> DeviceBatchLoader:
        # loop.py:312-315 + :1313-1317: epoch e (0-based) draws with seed base_seed + e + 1
        return DeviceBatchLoader(train_ds, batch_size, shuffle=True, seed=base_seed + max(0, int(epoch_idx)),
                                 bucket_batching=bool(cfg.get("bucket_batching", False)),
                                 n_buckets=int(cfg.get("n_buckets", 8)), rank=rank, world=world)

    def val_loader() -> DeviceBatchLoader:
        # every val batch exactly once over the ranks (sums reduced after the pass)
        return DeviceBatchLoader(val_ds, batch_size, shuffle=False, rank=rank, world=world, drop_remainder=False)

    multi_offset_weights = (normalize_offset_weights([int(x) for x in cfg.get("multi_offset_targets", [])],
                                                     cfg.get("multi_offset_weights"))
                            if bool(cfg.get("multi_offset_loss_enabled", False)) else {})
    term_enabled = bool(cfg.get("termination_loss_enabled", False))
    term_weight = float(cfg.get("termination_loss_weight", 0.1))
    term_stop_ids = tuple(int(x) for x in cfg.get("termination_stop_ids", [2]))
    term_edges = tuple(int(x) for x in cfg.get("termination_bucket_edges", [0, 3, 10, 30]))
    term_n_classes = int(cfg.get("termination_n_classes", len(term_edges) + 1))
    if term_n_classes != len(term_edges) + 1:
        raise ValueError("termination_n_classes must equal len(termination_bucket_edges) + 1")
    term_cw_values = cfg.get("termination_class_weights")
    if term_cw_values is not None:
        if len(term_cw_values) != term_n_classes:
            raise ValueError("termination_class_weights must contain termination_n_classes values")
        if any(float(v) <= 0 for v in term_cw_values):
            raise ValueError("termination_class_weights values must be positive")

    run_id = (getattr(args, "run_id", None) or cfg.get("run_id") or os.environ.get(RUN_ID_ENV) or "").strip() or None
    if not run_id:
        run_id = _auto_run_id(cfg, getattr(args, "config", None))
    cfg["run_id"] = run_id
    run_dir = Path("runs") / run_id
    ckpt_dir, scores_dir = run_dir / "checkpoints", run_dir / "scores"
    accumulation_health = AccumulationHealth()
    if is_main:
        ckpt_dir.mkdir(parents=True, exist_ok=True)
        scores_dir.mkdir(parents=True, exist_ok=True)
        vocab_tokens = itos if itos is not None else [f"token_{i}" for i in range(vocab_size)]
        (run_dir / "itos.txt").write_text("\n".join(vocab_tokens) + "\n")
    tokens_sha = hashlib.sha256("\n".join(itos or []).encode()).hexdigest() if itos else None
    cfg["itos_path"] = str(run_dir / "itos.txt")
    cfg["vocabulary"] = {"size": int(vocab_size), "sha256": tokens_sha, "legacy_adaptation": False}
    if is_main:
        (run_dir / "vocabulary.json").write_text(json.dumps(cfg["vocabulary"], indent=2, sort_keys=True) + "\n")
        config_src = getattr(args, "config", None)
        if config_src and os.path.isfile(config_src):
            shutil.copy2(config_src, ckpt_dir / "config.yaml")

    def write_failure_meta(exc: Exception) -> None:
        if is_main:
            write_meta(ckpt_dir, {"run_id": run_id, "status": "failed", "error_type": type(exc).__name__,
                                  "error": str(exc), "accumulation_health": accumulation_health.metrics_dict(),
                                  "model_spec": {}})

    log_csv = Path(cfg["log_csv"]) if cfg.get("log_csv") else scores_dir / "curves.csv"
    if not log_csv.is_absolute() and cfg.get("log_csv"):
        log_csv = (scores_dir / log_csv).resolve()
    is_resume_csv = resume_path is not None and log_csv.exists()
    if is_main and not is_resume_csv:
        log_csv.parent.mkdir(parents=True, exist_ok=True)
        with log_csv.open("w", newline="") as f:
            offset_cols = []
            for o in sorted(multi_offset_weights):
                offset_cols += [f"train_offset_{o}", f"val_offset_{o}"]
            term_cols = ["train_term_loss", "val_term_loss"] if term_enabled else []
            csv.writer(f).writerow(["step", "train_loss", "val_loss", "train_next_loss", "val_next_loss",
                                    "perplexity", "lr", *offset_cols, *term_cols])

    torch.manual_seed(base_seed)
    model = build_model(cfg, device)
    model._seed_rank = rank  # independent dropout masks per rank
    if transfer_path:  # loop.py:824-877
        if is_main:
            print(f"[transfer] initializing model from {transfer_path}")
        ck_t = torch.load(transfer_path, map_location=device, weights_only=True)
        sd = ck_t["model"] if isinstance(ck_t, dict) and "model" in ck_t else ck_t
        t_cfg = ck_t.get("cfg", {}) if isinstance(ck_t, dict) else {}
        source_itos = transfer_source_itos(transfer_path, t_cfg)
        report = load_transfer_state_dict(model, sd, source_itos=source_itos,
                                          target_itos=itos if itos is not None else None)
        src_rows = int(sd["tok_emb.weight"].shape[0]) if "tok_emb.weight" in sd else None
        cfg["vocabulary"]["legacy_adaptation"] = bool(src_rows != vocab_size or report["loaded_rows"])
        cfg["vocabulary"]["transfer"] = {"checkpoint": str(transfer_path), "source_embedding_rows": src_rows,
                                         "source_tokenizer_entries": len(source_itos) if source_itos else None,
                                         "target_vocab_size": int(vocab_size), "loaded_rows": report["loaded_rows"],
                                         "skipped": report["skipped"]}
        if is_main:
            (run_dir / "vocabulary.json").write_text(json.dumps(cfg["vocabulary"], indent=2, sort_keys=True) + "\n")
            print(f"[transfer] loaded_exact={len(report['loaded_exact'])} row_loaded={report['loaded_rows']}")
            if report["skipped"]:
                print(f"[transfer] skipped_shape_or_missing={report['skipped']}")
            if report["missing"]:
                print(f"[transfer] missing_after_adapt={report['missing']}")
            if report["unexpected"]:
                print(f"[transfer] unexpected_after_adapt={report['unexpected']}")
    term_cw = (torch.tensor([float(v) for v in term_cw_values], dtype=torch.float32, device=device)
               if term_cw_values is not None else None)
    lr_base = float(cfg.get("lr", 5e-6))
    optim = FusedAdamW(model, lr=lr_base, weight_decay=float(cfg.get("weight_decay", 0.05)),
                       lr_embedding=float(cfg.get("lr_embedding", lr_base)))
    scheduler_name = str(cfg.get("scheduler", "cosine")).lower()
    if scheduler_name not in {"cosine", "plateau"}:
        scheduler_name = "cosine"
    gacc = int(cfg.get("grad_accum_steps", 16))
    max_nonfinite_groups = int(cfg.get("max_nonfinite_accumulation_groups", 3))
    if max_nonfinite_groups < -1:
        raise ValueError("max_nonfinite_accumulation_groups must be -1 or greater")
    min_lr = float(cfg.get("min_lr", 1e-5))
    base_lr = float(cfg["lr"])
    n_params = sum(p.numel() for p in model.parameters())
    epochs_cfg = cfg.get("epochs", 5)
    if isinstance(epochs_cfg, str) and epochs_cfg.strip().lower() == "auto":
        tokens_target = max(1.0, float(cfg.get("tokens_per_param", 20.0)) * float(n_params))
        tokens_per_epoch = max(1.0, float(len(train_ds) * cfg["block_size"]))
        est = int(math.ceil(tokens_target / tokens_per_epoch))
        max_epochs = max(int(cfg.get("epochs_min", 1)), min(est, int(cfg.get("epochs_max", max(1, est)))))
    else:
        max_epochs = int(epochs_cfg)
    probe_loader = train_loader_for(0)
    train_batches = len(probe_loader)
    steps_per_epoch = math.ceil(train_batches / max(1, gacc))
    total_steps = int(cfg.get("scheduler_total_steps", max(1, steps_per_epoch * max_epochs)))
    if total_steps <= 0:
        raise ValueError("scheduler_total_steps must be positive")
    warmup_steps = resolve_warmup_steps(cfg, total_steps)
    cfg["resolved_warmup_steps"] = warmup_steps
    use_cosine = scheduler_name == "cosine"
    if use_cosine:
        scheduler = torch.optim.lr_scheduler.LambdaLR(optim, cosine_lr_lambda(warmup_steps, total_steps, base_lr,
                                                                              min_lr))
    else:
        scheduler = torch.optim.lr_scheduler.ReduceLROnPlateau(optim, mode="min", factor=0.5,
                                                               patience=cfg.get("plateau_patience", 2),
                                                               min_lr=min_lr)
    run_fingerprint = configuration_fingerprint(cfg)

    st = SimpleNamespace(start_epoch=0, best=float("inf"), no_improve=0, step=0, consumed=0, pending_tokens=None,
                         best_epoch=None, resume_mb=0, cur_epoch=0, cur_mb=0, cur_resume_mb=0)
    epoch_metrics = {"total_loss_sum": 0.0, "next_loss_sum": 0.0, "microbatches": 0, "initial_loss": None}
    pending_metrics = dict(epoch_metrics)

    if resume_path:
        ck = torch.load(resume_path, map_location=device, weights_only=True)
        model.load_state_dict(ck["model"])
        if "optimizer" in ck:
            try:
                optim.load_state_dict(ck["optimizer"])
            except Exception as exc:  # reference: warn and continue (loop.py:889-893)
                print(f"[resume] optimizer state load failed: {exc}")
        if ck.get("scheduler") is not None:
            try:
                scheduler.load_state_dict(ck["scheduler"])
            except Exception as exc:
                print(f"[resume] scheduler state load failed: {exc}")
        restore_rng_state(ck.get("rng_state"))
        if "dropout_seed" in ck:
            model._dropout_seed = int(ck["dropout_seed"])
        st.start_epoch = int(ck.get("epoch", 0))
        st.step = int(ck.get("step", 0))
        st.consumed = int(ck.get("consumed_train_tokens", 0))
        st.best = float(ck.get("best_val", st.best))
        st.best_epoch = ck.get("best_epoch")
        st.no_improve = int(ck.get("no_improve", 0))
        st.resume_mb = int(ck.get("epoch_microbatch_idx", 0) or 0)
        accumulation_health.load_state_dict(ck.get("accumulation_health"))
        for k in epoch_metrics:
            if k in (ck.get("epoch_train_metrics") or {}):
                epoch_metrics[k] = ck["epoch_train_metrics"][k]
        if ck.get("batch_size") is not None and int(ck["batch_size"]) != batch_size:
            st.resume_mb = 0
        if ck.get("grad_accum_steps") is not None and int(ck["grad_accum_steps"]) != gacc:
            st.resume_mb = 0

    every_steps = int(cfg.get("checkpoint_every_steps", 0) or 0)
    every_minutes = float(cfg.get("checkpoint_every_minutes", 0.0) or 0.0)
    last_saved = {"step": st.step, "t": time.monotonic()}

    def payload(epoch_idx, train_loss=float("inf"), val_loss=float("inf"), train_next_loss=None,
                val_next_loss=None, train_term_loss=None, val_term_loss=None) -> dict:
        done = val_loss != float("inf")
        return {
            "model": model.state_dict(), "optimizer": optim.state_dict(),
            "scheduler": scheduler.state_dict() if scheduler is not None else None, "cfg": _plain(cfg),
            "epoch": epoch_idx if done else max(0, epoch_idx - 1), "val_loss": val_loss, "train_loss": train_loss,
            "train_next_loss": train_next_loss, "val_next_loss": val_next_loss, "train_term_loss": train_term_loss,
            "val_term_loss": val_term_loss, "train_replay_term_loss": None, "best_val": st.best,
            "best_epoch": st.best_epoch, "no_improve": st.no_improve, "step": st.step,
            "consumed_train_tokens": int(st.consumed), "runtime_memory": {},
            "epoch_microbatch_idx": 0 if done else int(st.cur_resume_mb),
            "last_seen_microbatch_idx": int(st.cur_mb), "batch_size": batch_size, "grad_accum_steps": gacc,
            "train_examples": int(len(train_ds)), "train_batches": int(train_batches),
            "accumulation_health": accumulation_health.state_dict(),
            "max_nonfinite_accumulation_groups": max_nonfinite_groups, "epoch_train_metrics": dict(epoch_metrics),
            "run_progress": {"completed_epochs": epoch_idx if done else max(0, epoch_idx - 1),
                             "current_epoch": epoch_idx, "microbatch": 0 if done else int(st.cur_resume_mb),
                             "optimizer_step": st.step},
            "rng_state": capture_rng_state(), "run_fingerprint": run_fingerprint,
            "dropout_seed": int(model._dropout_seed),
        }

    def save(p: dict, name: str) -> None:
        if is_main:
            save_checkpoint_atomic(p, ckpt_dir / name)

    dp = DataParallelStep(model, optim) if world > 1 else None
    wall_limit = cfg.get("max_time_minutes")
    t_wall0 = time.perf_counter()
    ctl = GroupController(gacc=gacc, health=accumulation_health, world=world, group=ctrl,
                          wall_limit_s=float(wall_limit) * 60.0 if wall_limit else None, t0=t_wall0)
    # class weights of the next-codon loss, once (the reference checks torch.all(w == 1) per step)
    offset_lw = model.loss_weights if not bool(torch.all(model.loss_weights == 1.0)) else None
    offset_keys = sorted(multi_offset_weights)
    stats_host = torch.empty(4 + 2 * len(offset_keys), dtype=torch.float32, pin_memory=True)

    def forward_objective(xb, yb):
        """The trainer's objective (loop.py:1075-1112) as device tensors: (total, next, term or
        None, {offset: loss}, {offset: n_valid})."""
        need_aux = term_enabled or bool(multi_offset_weights)
        if need_aux:
            logits, next_loss, aux = model(xb, yb, return_aux=True)
        else:
            logits, next_loss = model(xb, yb)
            aux = {}
        total = next_loss
        offset_losses, offset_counts = {}, {}
        if multi_offset_weights:
            off_total, offset_losses, offset_counts = obj.multi_offset_lm_loss(
                aux.get("offset_logits", logits), yb, multi_offset_weights,
                label_smoothing=float(cfg.get("label_smoothing", 0.0)), loss_weights=offset_lw, return_counts=True)
            total = total + off_total
        term_loss = None
        if term_enabled:
            labels = obj.termination_distance_bucket_labels(yb, stop_ids=term_stop_ids, bucket_edges=term_edges)
            term_loss = obj.termination_aux_loss(aux["termination_logits"], labels, class_weights=term_cw)
            total = total + term_weight * term_loss
        return total, next_loss, term_loss, offset_losses, offset_counts

    def read_stats(total, next_loss, term_loss, off_losses, off_counts, yb):
        """One device->host transfer of the microbatch's scalars, recorded right after the
        forward: the caller enqueues the backward and then waits on the returned event only,
        so the backward's kernels run while the host decides."""
        parts = [total.detach().float().reshape(1), next_loss.detach().float().reshape(1),
                 (term_loss.detach().float() if term_loss is not None else torch.zeros((), device=device)).reshape(1),
                 yb.ne(PAD_ID).sum().reshape(1).float()]
        for k in offset_keys:
            parts.append(off_losses[k].detach().float().reshape(1) if k in off_losses
                         else torch.zeros(1, device=device))
            parts.append(off_counts[k].float().reshape(1) if k in off_counts else torch.zeros(1, device=device))
        host = stats_host[: len(parts)]
        host.copy_(torch.cat(parts), non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        return host, ev

    def unpack(host):
        v = host.tolist()
        total, nxt, term, ntok = v[0], v[1], v[2], v[3]
        offs = {}
        for i, k in enumerate(offset_keys):  # offsets without a valid target are skipped
            if v[5 + 2 * i] > 0:
                offs[k] = v[4 + 2 * i]
        return total, nxt, term, int(round(ntok)), offs

    def one_pass(split, loader, epoch_idx, skip=0):
        train = split == "train"
        model.train(train)
        if train:
            total, next_total, n = (float(epoch_metrics["total_loss_sum"]), float(epoch_metrics["next_loss_sum"]),
                                    int(epoch_metrics["microbatches"]))
        else:
            total, next_total, n = 0.0, 0.0, 0
        term_total, term_count = 0.0, 0
        off_tot = {o: 0.0 for o in multi_offset_weights}
        off_cnt = {o: 0 for o in multi_offset_weights}
        optim.zero_grad(set_to_none=True)
        skipped = 0
        health_before = accumulation_health.state_dict()
        pending = {"tok": 0}
        handles: list = []

        def drain():
            for h in handles:
                h.wait()
            handles.clear()

        def step_optimizer(group_size: int, batch_idx: int) -> None:
            if group_size <= 0:
                return
            if world > 1:
                if handles:
                    drain()  # the buckets were all-reduced during this microbatch's backward
                else:
                    dist.all_reduce(model.flat_grads(), op=dist.ReduceOp.SUM)
            if (not use_cosine) and warmup_steps > 0 and st.step < warmup_steps:
                for pg in optim.param_groups:
                    pg["lr"] = base_lr * float(st.step + 1) / max(1, warmup_steps)
            optim.step(grad_scale=1.0 / (group_size * world))
            optim.zero_grad(set_to_none=True)
            accumulation_health.complete_group()
            st.consumed += int(round(ctl.sum([pending["tok"]])[0]))
            pending["tok"] = 0
            for k in ("total_loss_sum", "next_loss_sum", "microbatches"):
                epoch_metrics[k] += pending_metrics[k]
            if epoch_metrics["initial_loss"] is None:
                epoch_metrics["initial_loss"] = pending_metrics["initial_loss"]
            pending_metrics.update(total_loss_sum=0.0, next_loss_sum=0.0, microbatches=0, initial_loss=None)
            st.step += 1
            st.cur_resume_mb = batch_idx + 1
            if use_cosine:
                scheduler.step()

        shard = len(loader)
        batch_idx = -1
        for batch_idx, (xb, yb) in enumerate(loader):
            st.cur_epoch = epoch_idx
            if train and batch_idx < skip:
                st.cur_mb = st.cur_resume_mb = batch_idx + 1
                continue
            st.cur_mb = batch_idx + 1
            with torch.set_grad_enabled(train):
                loss, next_loss, term_loss, off_losses, off_counts = forward_objective(xb, yb)
            host, ev = read_stats(loss, next_loss, term_loss, off_losses, off_counts, yb)
            if train:
                # backward enqueued before the finiteness verdict: a nonfinite microbatch aborts
                # its whole group, whose gradients are then discarded anyway (loop.py:1197-1219)
                if dp is not None and ctl.completes_group(batch_idx == shard - 1):
                    model._bucket_hook = dp.bucket_hook(handles)
                loss.backward()
            ev.synchronize()
            vals = unpack(host)
            if train:
                abort, stop = ctl.agree(not math.isfinite(vals[0]))
            else:
                abort, stop = not math.isfinite(vals[0]), False
            if abort:  # torch.isfinite(loss), loop.py:1197
                skipped += 1
                if train:
                    drain()
                    discarded = accumulation_health.abort_group(optim)
                    pending["tok"] = 0
                    pending_metrics.update(total_loss_sum=0.0, next_loss_sum=0.0, microbatches=0, initial_loss=None)
                    st.cur_resume_mb = batch_idx + 1
                    if is_main:
                        print(f"[train] aborted nonfinite accumulation group at microbatch={batch_idx + 1}; "
                              f"discarded_finite_microbatches={discarded} "
                              f"aborted_groups={accumulation_health.aborted_groups}")
                    if accumulation_health.exceeds_limit(max_nonfinite_groups):
                        raise NonfiniteGroupLimitError(
                            "nonfinite accumulation groups exceeded configured maximum "
                            f"{max_nonfinite_groups}: {accumulation_health.aborted_groups}")
                continue
            stepped = False
            v_total, v_next, v_term, ntok, v_offs = vals
            if train:
                if epoch_metrics["initial_loss"] is None and pending_metrics["initial_loss"] is None:
                    pending_metrics["initial_loss"] = v_total
                pending_metrics["total_loss_sum"] += v_total
                pending_metrics["next_loss_sum"] += v_next
                pending_metrics["microbatches"] += 1
                pending["tok"] += ntok
                accumulation_health.record_finite_microbatch()
                if accumulation_health.active_microbatches == gacc:
                    step_optimizer(accumulation_health.active_microbatches, batch_idx)
                    stepped = True
            else:
                total += v_total
                next_total += v_next
            if term_loss is not None:
                term_total += v_term
                term_count += 1
            for o, val in v_offs.items():
                off_tot[o] += val
                off_cnt[o] += 1
            n += 1
            if stepped and is_main and (
                    (every_steps > 0 and st.step - last_saved["step"] >= every_steps) or
                    (every_minutes > 0 and time.monotonic() - last_saved["t"] >= every_minutes * 60)):
                p = payload(epoch_idx)
                p["checkpoint_reason"] = "periodic"
                save(p, "last.pt")
                last_saved.update(step=st.step, t=time.monotonic())
            if stop:
                raise WallTimeLimitException()
        if train and accumulation_health.active_microbatches:
            step_optimizer(accumulation_health.active_microbatches, batch_idx)
        drain()
        if train:
            total, next_total, n = (float(epoch_metrics["total_loss_sum"]), float(epoch_metrics["next_loss_sum"]),
                                    int(epoch_metrics["microbatches"]))
        elif world > 1:
            total, next_total, n, term_total, term_count = ctl.sum([total, next_total, n, term_total, term_count])
            for o in off_tot:
                off_tot[o], off_cnt[o] = ctl.sum([off_tot[o], off_cnt[o]])
        offset_avgs = {o: off_tot[o] / max(off_cnt[o], 1) for o in off_tot}
        health_after = accumulation_health.state_dict()
        return (total / max(n, 1), next_total / max(n, 1),
                (term_total / max(term_count, 1)) if term_enabled else None, skipped, offset_avgs,
                {k: health_after[k] - health_before[k] for k in health_after})

    history = []
    try:
        for epoch in range(st.start_epoch, max_epochs):
            epoch_idx = epoch + 1
            skip = st.resume_mb if epoch == st.start_epoch else 0
            st.resume_mb = 0
            if skip == 0:
                epoch_metrics.update(total_loss_sum=0.0, next_loss_sum=0.0, microbatches=0, initial_loss=None)
                pending_metrics.update(total_loss_sum=0.0, next_loss_sum=0.0, microbatches=0, initial_loss=None)
            tr_loss, tr_next, tr_term, tr_skips, tr_offs, tr_health = one_pass("train", train_loader_for(epoch + 1),
                                                                               epoch_idx, skip)
            with torch.no_grad():
                va_loss, va_next, va_term, va_skips, va_offs, _ = one_pass("val", val_loader(), epoch_idx)
            ppl = math.exp(min(20.0, va_next))
            if not use_cosine:
                scheduler.step(va_loss)
            lr_now = optim.param_groups[0]["lr"]
            if is_main:
                msg = (f"[epoch {epoch_idx}] train {tr_loss:.3f} | val {va_loss:.3f} | next_val {va_next:.3f} "
                       f"| ppl {ppl:.2f} | lr {lr_now:.2e}")
                if tr_skips or va_skips:
                    msg += f" | skips train={tr_skips} val={va_skips}"
                print(msg)
            improved = va_loss + 1e-6 < st.best
            if improved:
                st.best, st.best_epoch, st.no_improve = va_loss, epoch_idx, 0
            else:
                st.no_improve += 1
            p = payload(epoch_idx, tr_loss, va_loss, tr_next, va_next, tr_term, va_term)
            save(p, "last.pt")
            last_saved.update(step=st.step, t=time.monotonic())
            if cfg.get("save_epochs", False):
                save(p, f"epoch_{epoch_idx}.pt")
            if is_main:
                with log_csv.open("a", newline="") as f:
                    row = [epoch_idx, f"{tr_loss:.4f}", f"{va_loss:.4f}", f"{tr_next:.4f}", f"{va_next:.4f}",
                           f"{ppl:.3f}", f"{lr_now:.3e}"]
                    for o in sorted(multi_offset_weights):
                        row += [f"{tr_offs.get(o, 0.0):.4f}", f"{va_offs.get(o, 0.0):.4f}"]
                    if term_enabled:
                        row += [f"{tr_term:.4f}", f"{va_term:.4f}"]
                    csv.writer(f).writerow(row)
            history.append({"epoch": epoch_idx, "train_loss": tr_loss, "val_loss": va_loss,
                            "train_next_loss": tr_next, "val_next_loss": va_next, "train_term_loss": tr_term,
                            "val_term_loss": va_term, "train_replay_term_loss": None, "perplexity": ppl,
                            "lr": lr_now, "nonfinite_microbatches": tr_health["nonfinite_microbatches"],
                            "aborted_accumulation_groups": tr_health["aborted_groups"],
                            "discarded_finite_microbatches": tr_health["discarded_finite_microbatches"]})
            if improved:
                save(p, "best.pt")
                save(p, f"best_epoch_{epoch_idx:03d}.pt")
            elif int(cfg.get("early_stop_patience", 5)) > 0 and st.no_improve >= int(cfg.get("early_stop_patience", 5)):
                if is_main:
                    print("[early-stopping] no improvement; stopping.")
                break
    except NonfiniteGroupLimitError as exc:
        p = payload(st.cur_epoch or (st.start_epoch + 1))
        p["checkpoint_reason"] = "nonfinite_group_limit"
        save(p, "last.pt")
        write_failure_meta(exc)
        raise
    except WallTimeLimitException:
        p = payload(st.cur_epoch or (st.start_epoch + 1))
        p["checkpoint_reason"] = "wall_time"
        save(p, "last.pt")
        _finish(is_main, ckpt_dir, scores_dir, run_id, t_wall0, st, accumulation_health, model, history, "stopped")
        return
    except Exception as exc:
        if _is_oom(exc):  # loop.py:1501-1549: save last.pt, halve batch_size in the YAML, re-raise
            _oom_safeguard(exc, is_main, lambda: payload(st.cur_epoch or (st.start_epoch + 1)), save,
                           getattr(args, "config", None), cfg.get("primary_training_contract") is not None)
            raise
        write_failure_meta(exc)
        raise
    _finish(is_main, ckpt_dir, scores_dir, run_id, t_wall0, st, accumulation_health, model, history, "completed")


def _is_oom(exc: Exception) -> bool:
    """The reference's test on the message (loop.py:1501-1502): HIP/torch allocation failures."""
    s = str(exc).lower()
    return "out of memory" in s or "oom" in s or "allocate" in s or "allocation" in s


def _oom_safeguard(exc, is_main, make_payload, save, config_path, primary) -> None:
    """OOM safeguard of loop.py:1503-1549: checkpoint last.pt with checkpoint_reason "oom", then
    (unless the config is an immutable primary contract) rewrite the YAML with batch_size halved
    and grad_accum_steps doubled so the next launch fits; the caller re-raises."""
    if not is_main:
        return
    print("\n" + "=" * 80)
    print("[OOM SAFEGUARD] Out-Of-Memory error detected during training loop execution!")
    print(f"Error detail: {exc}")
    print("Attempting to save last.pt checkpoint and downscale batch size in the config..." if not primary
          else "Attempting to save last.pt without modifying the immutable config...")
    print("=" * 80 + "\n")
    try:
        p = make_payload()
        p["checkpoint_reason"] = "oom"
        save(p, "last.pt")
        print("[OOM SAFEGUARD] Gracefully saved checkpoint to last.pt.")
    except Exception as save_exc:
        print(f"[OOM SAFEGUARD] Failed to save checkpoint: {save_exc}")
    if primary:
        print("[OOM SAFEGUARD] Immutable primary config was not modified; "
              "a new versioned runtime contract is required to change batch size.")
        return
    if not config_path or not os.path.isfile(config_path):
        return
    try:
        import yaml
        with open(config_path) as f:
            data = yaml.safe_load(f) or {}
        old_bs, old_gas = data.get("batch_size", 4), data.get("grad_accum_steps", 32)
        data["batch_size"], data["grad_accum_steps"] = max(1, old_bs // 2), old_gas * 2
        with open(config_path, "w") as f:
            yaml.safe_dump(data, f)
        print(f"[OOM SAFEGUARD] Config file {config_path} batch_size downscaled: {old_bs} -> {data['batch_size']} "
              f"(grad_accum_steps doubled: {old_gas} -> {data['grad_accum_steps']})")
    except Exception as yml_exc:
        print(f"[OOM SAFEGUARD] Failed to update config: {yml_exc}")


def _finish(is_main, ckpt_dir, scores_dir, run_id, t_wall0, st, health, model, history, status):
    if not is_main:
        return
    meta = {"run_id": run_id, "train_wall_sec": round(time.perf_counter() - t_wall0, 2),
            "best_epoch": st.best_epoch, "best_val_loss": float(st.best) if st.best != float("inf") else None,
            "status": status, "accumulation_health": health.state_dict(), "model_spec": model.to_dict()}
    if history:
        h = history[-1]
        meta.update({"last_epoch": h["epoch"], "last_val_loss": h["val_loss"], "last_train_loss": h["train_loss"],
                     "last_val_next_loss": h["val_next_loss"], "last_train_next_loss": h["train_next_loss"],
                     "last_val_term_loss": h["val_term_loss"], "last_train_term_loss": h["train_term_loss"],
                     "last_train_replay_term_loss": None, "last_perplexity": h["perplexity"]})
        (scores_dir / "metrics.json").write_text(json.dumps(meta, indent=2) + "\n")
    write_meta(ckpt_dir, meta)


__all__ = ["run_training", "AccumulationHealth", "NonfiniteGroupLimitError", "resolve_warmup_steps",
           "normalize_offset_weights", "cosine_lr_lambda", "build_model", "save_checkpoint_atomic"]
