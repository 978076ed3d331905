#!/usr/bin/env python3
"""Sequence embeddings from a trained codon LM on the MI355X (mirrors scripts/extract_embeddings.py).

    python -m codonlm_amd.extract_embeddings --run_dir runs/<ID> --fasta genes.fasta --out emb.npz \
        [--hidden-layers 0,6,final] [--pooling-modes mean_nonpad,mean_content,eos] [--batch-size 16]

Same CLI, tokenisation (BOS + codons + EOS, unknown codons dropped, right-truncated at
block_size), batching with right PAD, hidden-layer / pooling-mode selection, NPZ arrays
(``X__layer_{k}__{mode}``, ``X`` when one representation is asked for, ``ids``) and
metadata JSON keys as the reference (:173-409).  What runs differs: one native engine
forward per batch on the GPU, and the pooling reads the engine's hidden-state buffers in
place (cg_pool_hidden) -- no (B, T, d) copies leave HBM.  ``--dtype bf16`` selects the
throughput engine; the default fp32 is the reference's arithmetic.

``--manifest`` binds a frozen dataset manifest exactly as the reference (:227-230, the
``provenance`` module): the manifest is validated, and a corrected checkpoint must name the same
dataset and vocabulary; without it such a checkpoint is refused.  Not supported (outside the hot
path): shape-guided checkpoints.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import subprocess
from datetime import datetime, timezone
from pathlib import Path
from typing import List, Tuple

import numpy as np
import torch

from . import ops
from .checkpoints import build_codon_model_from_cfg, build_model_from_state, load_codon_checkpoint
from .provenance import bind_checkpoint_dataset, bind_dataset_manifest

POOLING_MODES = ("mean_nonpad", "mean_content", "eos")


def read_fasta(path: Path) -> List[Tuple[str, str]]:
    """_read_fasta (:39-57)."""
    out, name, chunks = [], None, []
    for line in Path(path).read_text().splitlines():
        line = line.strip()
        if not line:
            continue
        if line.startswith(">"):
            if name is not None:
                out.append((name, "".join(chunks)))
            name, chunks = line[1:].strip(), []
        else:
            chunks.append(line)
    if name is not None:
        out.append((name, "".join(chunks)))
    return out


def dna_to_codon_tokens(dna: str) -> List[str]:
    """_dna_to_codon_tokens (:60-66)."""
    s = dna.strip().upper().replace("U", "T")
    n = (len(s) // 3) * 3
    return [s[i:i + 3] for i in range(0, n, 3)]


def load_itos(path: Path) -> tuple:
    """src/codonlm/training/vocabulary.py:62-79 (strict: no empty or duplicate tokens)."""
    path = Path(path)
    if not path.exists():
        raise RuntimeError(f"Tokenizer vocabulary not found: {path}")
    raw = path.read_text().splitlines()
    if not raw:
        raise RuntimeError(f"Tokenizer vocabulary is empty: {path}")
    tokens = tuple(t.strip() for t in raw)
    empty = [i for i, t in enumerate(tokens) if not t]
    if empty:
        raise RuntimeError(f"Tokenizer vocabulary contains empty token IDs {empty}: {path}")
    dups = sorted({t for t in tokens if tokens.count(t) > 1})
    if dups:
        raise RuntimeError(f"Tokenizer vocabulary contains duplicate tokens {dups}: {path}")
    return tokens


def _sha256(path: Path) -> str:
    h = hashlib.sha256()
    with Path(path).open("rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()


def _git_sha():
    try:
        return subprocess.run(["git", "rev-parse", "HEAD"], check=True, capture_output=True, text=True).stdout.strip()
    except (OSError, subprocess.CalledProcessError):
        return None


def validate_vocabulary(itos, state, cfg, path) -> None:
    """_validate_vocabulary (:133-155)."""
    rows = int(state["tok_emb.weight"].shape[0])
    if rows != len(itos):
        raise RuntimeError(f"checkpoint embedding rows={rows} do not match vocabulary size={len(itos)}")
    out_rows = int(state["head.weight"].shape[0])
    if out_rows != len(itos):
        raise RuntimeError(f"checkpoint output rows={out_rows} do not match vocabulary size={len(itos)}")
    configured = cfg.get("vocab_size")
    if configured is not None and int(configured) != len(itos):
        raise RuntimeError(f"checkpoint vocab_size={configured} does not match vocabulary size={len(itos)}")
    meta = cfg.get("vocabulary") or {}
    if not isinstance(meta, dict):
        raise RuntimeError("checkpoint vocabulary metadata must be a mapping")
    expected = meta.get("sha256")
    if expected and expected != _sha256(path):
        raise RuntimeError("checkpoint vocabulary hash does not match run itos.txt")


def tokenize(seqs, stoi, mode: str, max_T: int):
    """(:291-305) -> [(id, token ids)]."""
    bos, eos = stoi.get("<BOS_CDS>"), stoi.get("<EOS_CDS>")
    examples = []
    for sid, seq in seqs:
        codons = dna_to_codon_tokens(seq) if mode == "dna_cds" else [t for t in seq.strip().upper().split() if t]
        toks = []
        if bos is not None:
            toks.append(bos)
        toks.extend(stoi[c] for c in codons if c in stoi)
        if eos is not None:
            toks.append(eos)
        if toks:
            examples.append((sid, toks[:max_T]))
    return examples


@torch.no_grad()
def pooled_representations(model, ids_tensor, layers, modes, content_ids, pad: int) -> dict:
    """{(layer, mode): fp32 (B, d)} for one padded batch: one engine forward, pooling in place."""
    eng = model.engine
    eng.forward(ids_tensor, None, training=False)
    out = {}
    for layer in layers:
        which = model.n_layer + 1 if layer == "final" else int(layer)
        h = eng.hidden(which)
        for mode in modes:
            out[(layer, mode)] = ops.pool_hidden(h, ids_tensor, mode, content_ids, pad)
    return out


def main(argv=None) -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--run_id")
    ap.add_argument("--run_dir")
    ap.add_argument("--fasta")
    ap.add_argument("--csv")
    ap.add_argument("--seq_col", default="seq")
    ap.add_argument("--mode", choices=["dna_cds", "codon_tokens"], default="dna_cds")
    ap.add_argument("--manifest", type=Path, help="frozen dataset manifest (corrected checkpoints)")
    ap.add_argument("--batch-size", type=int, default=16)
    ap.add_argument("--random-init-seed", type=int)
    ap.add_argument("--hidden-layers", default="final")
    ap.add_argument("--pooling-modes", default="mean_nonpad")
    ap.add_argument("--dtype", choices=["fp32", "bf16"], default="fp32")
    ap.add_argument("--out", required=True)
    args = ap.parse_args(argv)
    if args.batch_size < 1:
        ap.error("--batch-size must be at least 1")
    layer_values = ["final" if v.strip() == "final" else int(v) for v in args.hidden_layers.split(",")]
    pooling_modes = [v.strip() for v in args.pooling_modes.split(",")]

    rd = Path(args.run_dir) if args.run_dir else Path("runs") / args.run_id
    itos_path = rd / "itos.txt"
    itos = load_itos(itos_path)
    stoi = {t: i for i, t in enumerate(itos)}
    state_dict, cfg, checkpoint_path = load_codon_checkpoint(rd)
    valid_layers = set(range(int(cfg["n_layer"]) + 1)) | {"final"}
    if not layer_values or any(v not in valid_layers for v in layer_values):
        ap.error(f"--hidden-layers must be drawn from {sorted(map(str, valid_layers))}")
    if not pooling_modes or any(m not in POOLING_MODES for m in pooling_modes):
        ap.error(f"--pooling-modes must be drawn from {sorted(POOLING_MODES)}")
    manifest_provenance = None
    if args.manifest is not None:
        _, manifest_provenance = bind_dataset_manifest(args.manifest)
    checkpoint_dataset = bind_checkpoint_dataset(cfg, manifest_provenance)
    validate_vocabulary(itos, state_dict, cfg, itos_path)
    device = torch.device("cuda", torch.cuda.current_device())
    if args.random_init_seed is None:
        model = build_model_from_state(state_dict, cfg, compute_dtype=args.dtype, device=device)
        model_initialization = {"kind": "trained_checkpoint"}
        weights_sha = _sha256(checkpoint_path)
    else:
        torch.manual_seed(args.random_init_seed)
        model = build_codon_model_from_cfg(cfg, compute_dtype=args.dtype, device=device)
        model.eval()
        contract = json.dumps({"architecture": {k: cfg.get(k) for k in (
            "vocab_size", "block_size", "n_layer", "n_head", "n_embd", "dropout", "tie_embeddings", "n_kv_head",
            "use_sdpa", "use_swiglu", "use_rope")}, "seed": args.random_init_seed}, sort_keys=True).encode()
        weights_sha = hashlib.sha256(contract).hexdigest()
        model_initialization = {"kind": "random", "seed": args.random_init_seed}

    seqs = []
    if args.fasta:
        seqs += read_fasta(Path(args.fasta))
    if args.csv:
        import csv
        with open(args.csv, newline="") as f:
            for row in csv.DictReader(f):
                seqs.append((row.get("id", f"row{len(seqs)}"), row[args.seq_col]))
    if not seqs:
        raise SystemExit("No sequences provided (use --fasta or --csv)")
    pad = stoi.get("<PAD>", 0)
    max_T = int(cfg.get("block_size", model.block_size))
    examples = tokenize(seqs, stoi, args.mode, max_T)
    content_ids = sorted(i for i, t in enumerate(itos) if len(t) == 3 and t.isalpha())
    vectors = {f"layer_{layer}__{mode}": [] for layer in layer_values for mode in pooling_modes}
    ids = []
    for start in range(0, len(examples), args.batch_size):
        batch = examples[start:start + args.batch_size]
        width = max(len(t) for _, t in batch)
        host = np.full((len(batch), width), pad, dtype=np.int64)
        for r, (_, toks) in enumerate(batch):
            host[r, :len(toks)] = toks
        ids_tensor = torch.from_numpy(host).to(device)
        reps = pooled_representations(model, ids_tensor, layer_values, pooling_modes, content_ids, pad)
        for (layer, mode), t in reps.items():
            vectors[f"layer_{layer}__{mode}"].extend(t.cpu().numpy())
        ids.extend(sid for sid, _ in batch)
    if not ids:
        raise SystemExit("No valid sequences after tokenization")

    out_path = Path(args.out)
    out_path.parent.mkdir(parents=True, exist_ok=True)
    arrays = {f"X__{name}": np.stack(v, axis=0) for name, v in vectors.items()}
    if len(arrays) == 1:
        arrays["X"] = next(iter(arrays.values()))
    np.savez_compressed(out_path, **arrays, ids=np.array(ids, dtype=object))
    inputs = [Path(p) for p in (args.fasta, args.csv) if p]
    metadata = {
        "schema_version": 1, "validation_status": "causal_verified",
        "created_at": datetime.now(timezone.utc).isoformat(),
        "checkpoint": {"path": str(Path(checkpoint_path).resolve()), "sha256": _sha256(checkpoint_path)},
        "model_weights": {"sha256": weights_sha, "initialization": model_initialization},
        "dataset_manifest": manifest_provenance or {"status": "legacy_unverified"},
        "checkpoint_dataset": checkpoint_dataset,
        "vocabulary": {"path": str(itos_path.resolve()), "size": len(itos), "sha256": _sha256(itos_path)},
        "inputs": [{"path": str(p.resolve()), "sha256": _sha256(p)} for p in inputs],
        "mask_mode": "canonical_causal_segment" if model.sep_id is not None else "canonical_causal",
        "pooling_mode": ("mean_nonpad_including_special_tokens" if pooling_modes == ["mean_nonpad"]
                         else "multi_representation"),
        "representations": sorted(vectors), "shape_guidance": False, "block_size": max_T,
        "extraction_batch_size": args.batch_size, "truncation_policy": "right_truncate",
        "code_git_sha": _git_sha(),
    }
    out_path.with_suffix(out_path.suffix + ".metadata.json").write_text(
        json.dumps(metadata, indent=2, sort_keys=True) + "\n")
    print(f"[extract] wrote {args.out} with arrays={ {k: list(a.shape) for k, a in arrays.items()} }")


if __name__ == "__main__":
    main()
