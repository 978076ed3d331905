"""Transfer warm start with vocabulary remapping (mirrors src/codonlm/training/checkpoint.py).

``load_transfer_state_dict`` follows ``_load_transfer_state_dict`` (checkpoint.py:16-85):
for every tensor of the target model's state_dict,

* same shape and no token remap needed -> copied as is;
* same trailing shape but a different row count, or a vocabulary-row tensor
  (``tok_emb.weight`` / ``head.weight`` / ``loss_weights``) whose source and target itos
  differ -> the target's rows are kept and overwritten row by row: by token (target row of
  token t <- source row of token t) when both itos lists are known, otherwise the leading
  min(rows) rows;
* anything else is skipped.

The adapted tensors go through ``model.load_state_dict(strict=False)``; on the MI355X model
that writes the flat fp32 master buffer (and refreshes the bf16 shadow and loss weights).
"""
from __future__ import annotations

from pathlib import Path

import torch

VOCAB_ROW_NAMES = frozenset({"tok_emb.weight", "head.weight", "loss_weights"})


def read_itos(path_value, base_dir: Path | None = None):
    """checkpoint.py:5-13: itos lines of an existing file (relative paths under base_dir), else None."""
    if not path_value:
        return None
    path = Path(str(path_value))
    if not path.is_absolute() and base_dir is not None:
        path = Path(base_dir) / path
    if not path.exists():
        return None
    return [line.strip() for line in path.read_text().splitlines() if line.strip()]


def _remap_rows(target: torch.Tensor, source: torch.Tensor, src_index: dict, dst_index: dict):
    merged = target.detach().clone()
    copied = 0
    if src_index and dst_index:
        for tok, dst in dst_index.items():
            src = src_index.get(tok)
            if src is None or src >= source.shape[0] or dst >= merged.shape[0]:
                continue
            merged[dst] = source[src].to(device=merged.device, dtype=merged.dtype)
            copied += 1
    else:
        copied = min(int(source.shape[0]), int(merged.shape[0]))
        merged[:copied] = source[:copied].to(device=merged.device, dtype=merged.dtype)
    return merged, copied


def load_transfer_state_dict(model, source_state: dict, *, source_itos=None, target_itos=None) -> dict:
    """Adapt ``source_state`` to ``model`` and load it; returns the reference's report dict
    (loaded_exact / loaded_rows "name:count" / skipped / missing / unexpected)."""
    src_index = {tok: i for i, tok in enumerate(source_itos or [])}
    dst_index = {tok: i for i, tok in enumerate(target_itos or [])}
    vocab_differs = bool(src_index and dst_index) and list(source_itos) != list(target_itos)
    adapted, exact, rows, skipped = {}, [], [], []
    for name, tgt in model.state_dict().items():
        src = source_state.get(name)
        if src is None:
            skipped.append(name)
            continue
        remap = name in VOCAB_ROW_NAMES and vocab_differs
        if tuple(src.shape) == tuple(tgt.shape) and not remap:
            adapted[name] = src
            exact.append(name)
            continue
        if (src.ndim >= 1 and tgt.ndim >= 1 and tuple(src.shape[1:]) == tuple(tgt.shape[1:])
                and (src.shape[0] != tgt.shape[0] or remap)):
            merged, copied = _remap_rows(tgt, src, src_index, dst_index)
            if copied:
                adapted[name] = merged
                rows.append(f"{name}:{copied}")
            else:
                skipped.append(name)
            continue
        skipped.append(name)
    missing, unexpected = model.load_state_dict(adapted, strict=False)
    return {"loaded_exact": exact, "loaded_rows": rows, "skipped": skipped, "missing": list(missing),
            "unexpected": list(unexpected)}


def transfer_source_itos(transfer_path, transfer_cfg: dict):
    """loop.py:829-839: the source itos from the checkpoint cfg's itos_path (relative to the
    working directory), else itos.txt next to the checkpoint or one directory up."""
    itos = read_itos((transfer_cfg or {}).get("itos_path"), Path.cwd())
    if itos is None:
        p = Path(transfer_path).resolve()
        for cand in (p.parent / "itos.txt", p.parent.parent / "itos.txt"):
            itos = read_itos(str(cand))
            if itos is not None:
                break
    return itos


__all__ = ["read_itos", "load_transfer_state_dict", "transfer_source_itos", "VOCAB_ROW_NAMES"]
