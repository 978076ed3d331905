#!/usr/bin/env python3
"""CLI of the MI355X codon-LM trainer (mirrors src/codonlm/train_codon_lm.py:37-62).

    python -m codonlm_amd.train_codon_lm --config cfg.yaml [--run_id ID] [--resume last.pt] ...

Multi-GPU: launch one process per GPU with torch.distributed.run; the process group is
initialised here over RCCL (backend "nccl") and the loop shards batches across ranks.
"""
from __future__ import annotations

import argparse
import os

import torch
import torch.distributed as dist
import yaml

from .training.loop import run_training


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", required=True)
    ap.add_argument("--run_id", default=None, help="Unique run id; falls back to $RUN_ID or config.run_id")
    ap.add_argument("--resume", default=None, help="Path to checkpoint to resume training from")
    ap.add_argument("--transfer_from", default=None,
                    help="Path to pre-trained weights to initialize model from (ignores optimizer/step state)")
    ap.add_argument("--train_npz", action="append", default=None, help="Training NPZ file (repeatable)")
    ap.add_argument("--val_npz", action="append", default=None, help="Validation NPZ file (repeatable)")
    ap.add_argument("--test_npz", action="append", default=None, help="Test NPZ file (repeatable)")
    ap.add_argument("--save_epochs", action="store_true", help="Save checkpoint at every epoch")
    ap.add_argument("--max_time_minutes", type=float, default=None, help="Override config max_time_minutes")
    args = ap.parse_args(argv)
    with open(args.config) as f:
        cfg = yaml.safe_load(f) or {}
    if "data" in cfg and isinstance(cfg["data"], dict):
        for k, v in cfg["data"].items():
            cfg.setdefault(k, v)
    cfg["save_epochs"] = args.save_epochs or cfg.get("save_epochs", False)
    if args.max_time_minutes is not None:
        cfg["max_time_minutes"] = float(args.max_time_minutes)
    started = False
    if int(os.environ.get("WORLD_SIZE", "1")) > 1 and not dist.is_initialized():
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
        dist.init_process_group("nccl")
        started = True
    try:
        run_training(cfg, args)
    finally:
        if started:
            dist.destroy_process_group()


if __name__ == "__main__":
    main()
