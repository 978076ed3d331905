"""Termination / multi-offset auxiliary heads (model_tiny_gpt.py:329-337, objectives.py)."""


def aux_forward(model, idx, targets, attention_window):
    raise NotImplementedError("aux heads land with the C5 configuration")
