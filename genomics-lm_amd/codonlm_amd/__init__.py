"""codonlm_amd -- MI355X-native (gfx950) training/inference path for the genomics-lm codon LM.

Drop-in for src/codonlm/model_tiny_gpt.py (TinyGPT) and the codon trainer's hot loop,
backed by hand-written HIP kernels in libcodonlm_hip.so (include/codonlm_hip.h).
"""
from . import _lib  # noqa: F401  (fails loudly if the native library is missing)
from .model_tiny_gpt import TinyGPT, num_params  # noqa: F401

__all__ = ["TinyGPT", "num_params"]
