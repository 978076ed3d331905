"""Codon-LM training loop pieces for the MI355X path (mirrors src/codonlm/training)."""
