"""Shared pytest setup: repo-root + package paths, the `gpu` marker, golden loader."""
import json
import os
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
PKG = ROOT / "genomics-lm_amd"
for p in (str(ROOT), str(PKG)):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs under gpurun)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def load_golden(name):
    z = np.load(GOLDEN / f"{name}.npz", allow_pickle=False)
    d = {k: z[k] for k in z.files}
    cfg = json.loads(str(d.pop("config"))) if "config" in d else None
    return cfg, d


@pytest.fixture
def golden():
    return load_golden


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
