#!/usr/bin/env python3
"""Query a trained codon LM on the MI355X (mirrors scripts/query_model.py).

    python -m codonlm_amd.query_model <RUN_ID> --mode next --dna ATGAAACCC
    python -m codonlm_amd.query_model --run_dir runs/<ID> --mode generate --dna ATG --max_new 30 --topk 5
    python -m codonlm_amd.query_model <RUN_ID> --mode score --dna ATGAAATGA

Same modes, tokenisation (``dna_to_ids`` appends <EOS_CDS> even in ``next`` mode, :68-85),
context truncation to block_size, JSON answers (:253-295) and vocabulary / checkpoint
discovery as the reference.  ``dev()`` returns the MI355X (the reference's picks MPS/CPU,
:29-34) and every forward is the native engine; ``--dtype bf16`` selects the throughput
engine (default fp32 = the reference's arithmetic, greedy ids bit-exact).
"""
from __future__ import annotations

import argparse
import json
from pathlib import Path
from typing import Dict, List, Tuple

import numpy as np
import torch
import yaml

from .checkpoints import build_model_from_state as _build, load_codon_checkpoint
from .model_tiny_gpt import TinyGPT


def dev() -> torch.device:
    return torch.device("cuda", torch.cuda.current_device())


def _load_checkpoint(run_dir: Path) -> Tuple[Dict, Dict]:
    try:
        state_dict, cfg, _ = load_codon_checkpoint(run_dir)
    except FileNotFoundError:
        state_dict, cfg, _ = load_codon_checkpoint(Path("outputs/checkpoints") / run_dir.name)
    return state_dict, cfg


def _load_vocab(run_dir: Path) -> Tuple[List[str], Dict[str, int]]:
    itos_path = run_dir / "itos.txt"
    if not itos_path.exists():
        cfg_path = run_dir / "checkpoints" / "config.yaml"
        if cfg_path.exists():
            fallback = (yaml.safe_load(cfg_path.read_text()) or {}).get("itos_path")
            if fallback and Path(fallback).exists():
                itos_path = Path(fallback)
        if not itos_path.exists():
            raise FileNotFoundError(f"Missing itos.txt at {run_dir / 'itos.txt'} and no usable itos_path "
                                    "was found in checkpoints/config.yaml.")
    tokens = [ln.strip() for ln in itos_path.read_text().splitlines() if ln.strip()]
    return tokens, {t: i for i, t in enumerate(tokens)}


def _codon_ids(dna: str, stoi: Dict[str, int]) -> List[int]:
    dna = dna.strip().upper().replace("U", "T")
    out = []
    for i in range(0, len(dna) // 3 * 3, 3):
        idx = stoi.get(dna[i:i + 3])
        if idx is None:
            raise ValueError(f"Unknown codon: {dna[i:i + 3]}")
        out.append(idx)
    return out


def dna_to_ids(dna: str, stoi: Dict[str, int]) -> List[int]:
    """BOS + codons + EOS (:68-85)."""
    if len(dna.strip()) < 3:
        return []
    bos, eos = stoi.get("<BOS_CDS>"), stoi.get("<EOS_CDS>")
    return ([bos] if bos is not None else []) + _codon_ids(dna, stoi) + ([eos] if eos is not None else [])


def dna_prefix_to_ids(dna: str, stoi: Dict[str, int]) -> List[int]:
    """BOS + codons, no EOS (:88-104)."""
    if len(dna.strip()) < 3:
        return []
    bos = stoi.get("<BOS_CDS>")
    return ([bos] if bos is not None else []) + _codon_ids(dna, stoi)


def ids_to_codons(ids: List[int], itos: List[str]) -> List[str]:
    return [itos[i] if 0 <= i < len(itos) else f"<{i}>" for i in ids]


def build_model_from_state(state_dict: Dict, cfg: Dict, checkpoint=None, *, compute_dtype: str = "fp32",
                           device=None) -> TinyGPT:
    if bool(cfg.get("use_shape_guidance", False)):
        raise ValueError("shape-guided checkpoints are outside the MI355X hot path")
    return _build(state_dict, cfg, compute_dtype=compute_dtype, device=device if device is not None else dev())


@torch.no_grad()
def next_token(model: TinyGPT, device: torch.device, ctx_ids: List[int]) -> torch.Tensor:
    """logits[0, -1] of the (block_size-truncated) context (:160-182)."""
    max_T = getattr(model, "block_size", None)
    ids = ctx_ids[-max_T:] if max_T is not None else ctx_ids
    x = torch.tensor(ids, dtype=torch.long, device=device).unsqueeze(0)
    logits, _ = model(x)
    return logits[0, -1]


def _decode_loop(model: TinyGPT, device: torch.device, ctx_ids: List[int], max_new: int, pick,
                 eos_idx: int | None, kv_cache: bool) -> List[int]:
    """The autoregressive loop of query_model.py:185-214 with a KV cache: the prompt is prefilled
    once and each new token is one cached decode step (cg_model_decode) while the context fits
    block_size; once it does not, the reference's sliding-window re-forward takes over.
    ``pick(logits[V]) -> id`` chooses the next token."""
    ids = list(ctx_ids)
    max_T = getattr(model, "block_size", None)
    cache = None
    logits = None
    if kv_cache and max_T is not None and 0 < len(ids) < max_T:
        cache = model.engine.new_kv_cache(1, max_T)
        logits = cache.prefill(torch.tensor([ids], dtype=torch.long, device=device))[0, -1]
    for _ in range(max_new):
        if cache is None:
            logits = next_token(model, device, ids)
        next_id = int(pick(logits))
        ids.append(next_id)
        if max_T is not None and len(ids) > max_T:
            ids = ids[-max_T:]
        if eos_idx is not None and next_id == eos_idx:
            break
        if cache is not None:
            if cache.pos < cache.Tmax:
                logits = cache.decode(torch.tensor([next_id], device=device))[0]
            else:  # the context reached block_size: slide and recompute like the reference
                cache = None
    return ids


@torch.no_grad()
def generate(model: TinyGPT, device: torch.device, ctx_ids: List[int], max_new: int, temperature: float = 1.0,
             topk: int = 0, eos_idx: int | None = None, kv_cache: bool = True) -> List[int]:
    """Sampling loop of :185-214: temperature, optional top-k, torch.multinomial on the device
    RNG -- the same draws in the same order as the reference; the logits come from the KV cache
    (one decode step per token) instead of a full re-forward of the prefix."""
    def pick(logits):
        if temperature != 1.0:
            logits = logits / max(1e-6, float(temperature))
        probs = torch.softmax(logits, dim=-1)
        if topk and topk > 0:
            vals, idxs = torch.topk(probs, k=min(topk, probs.numel()))
            return idxs[torch.multinomial(vals, 1).item()].item()
        return torch.multinomial(probs, 1).item()
    return _decode_loop(model, device, ctx_ids, max_new, pick, eos_idx, kv_cache)


@torch.no_grad()
def greedy_generate(model: TinyGPT, device: torch.device, ctx_ids: List[int], max_new: int,
                    eos_idx: int | None = None, kv_cache: bool = True) -> List[int]:
    """Deterministic argmax continuation (the parity form of ``generate``), KV-cached the same way."""
    return _decode_loop(model, device, ctx_ids, max_new, lambda lg: torch.argmax(lg).item(), eos_idx, kv_cache)


@torch.no_grad()
def score_sequence(model: TinyGPT, device: torch.device, ids: List[int]) -> Dict[str, float]:
    x = torch.tensor(ids[:-1], dtype=torch.long, device=device).unsqueeze(0)
    y = torch.tensor(ids[1:], dtype=torch.long, device=device).unsqueeze(0)
    _, loss = model(x, y)
    loss_val = float(loss.item()) if loss is not None else float("nan")
    ppl = float(np.exp(min(20.0, loss_val))) if loss is not None else float("nan")
    return {"nll": loss_val, "ppl": ppl}


def _answer(dna: str, args, itos: List[str], stoi: Dict[str, int], model: TinyGPT, device: torch.device) -> Dict:
    ids = dna_to_ids(dna, stoi)
    if not ids:
        return {"error": "prompt too short (<3 nt)"}
    eos_idx = stoi.get("<EOS_CDS>")
    if args.mode == "next":
        probs = torch.softmax(next_token(model, device, ids), dim=-1)
        topv, topi = torch.topk(probs, k=min(args.topk, probs.numel()))
        return {"prompt": dna, "topk": [{"token": itos[i], "prob": float(p)}
                                        for p, i in zip(topv.tolist(), topi.tolist())]}
    if args.mode == "generate":
        gen = generate(model, device, ids, max_new=args.max_new, temperature=args.temperature,
                       topk=args.topk if args.topk > 0 else 0, eos_idx=eos_idx)
        return {"prompt": dna, "tokens": ids_to_codons(gen, itos)}
    if args.mode == "score":
        return score_sequence(model, device, ids)
    raise SystemExit(f"Unknown mode: {args.mode}")


def run_once(args) -> Dict:
    if getattr(args, "run_dir", None):
        rd = Path(args.run_dir)
        run_dir = rd if (rd / "itos.txt").exists() else (Path("runs") / rd.name)
    else:
        run_dir = Path("runs") / args.run_id
    itos, stoi = _load_vocab(run_dir)
    state_dict, cfg = _load_checkpoint(run_dir)
    device = dev()
    model = build_model_from_state(state_dict, cfg, compute_dtype=getattr(args, "dtype", "fp32"), device=device)
    if args.dna is None and not args.interactive:
        raise SystemExit("Provide --dna or use --interactive mode")
    if args.interactive:
        print("[interactive] enter DNA strings (CTRL+D to exit)")
        while True:
            try:
                line = input("> ").strip()
            except EOFError:
                break
            if line:
                print(json.dumps(_answer(line, args, itos, stoi, model, device), indent=2))
        return {}
    return _answer(args.dna, args, itos, stoi, model, device)


def main(argv=None) -> None:
    ap = argparse.ArgumentParser(description="Query a trained codon LM by run_id or run_dir.")
    ap.add_argument("run_id", nargs="?", help="Run identifier under runs/<RUN_ID>")
    ap.add_argument("--run_dir", help="Alternative to run_id; path to outputs/checkpoints/<RUN_ID> or runs/<RUN_ID>")
    ap.add_argument("--mode", choices=["next", "generate", "score"], default="next")
    ap.add_argument("--dna", help="DNA prompt (uppercase ACGT)")
    ap.add_argument("--topk", type=int, default=5)
    ap.add_argument("--temperature", type=float, default=1.0)
    ap.add_argument("--max_new", type=int, default=30)
    ap.add_argument("--interactive", action="store_true")
    ap.add_argument("--dtype", choices=["fp32", "bf16"], default="fp32")
    ap.add_argument("--out", help="optional JSON output path")
    args = ap.parse_args(argv)
    if not args.run_id and not args.run_dir:
        ap.error("provide either run_id or --run_dir")
    if args.run_id and args.run_dir:
        print("[warn] both run_id and --run_dir provided; using --run_dir")
        args.run_id = None
    result = run_once(args)
    if args.out:
        outp = Path(args.out)
        outp.parent.mkdir(parents=True, exist_ok=True)
        outp.write_text(json.dumps(result, indent=2) + "\n")
    elif result:
        print(json.dumps(result, indent=2))


if __name__ == "__main__":
    main()
