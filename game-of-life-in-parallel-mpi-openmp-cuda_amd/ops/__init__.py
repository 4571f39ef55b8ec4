"""Kernel-level ops (native HIP/CPU) and PyTorch/NumPy oracles."""
from .life_ops import life_step, life_step_numpy, life_step_torch, random_grid, rule_words

__all__ = ["life_step", "life_step_numpy", "life_step_torch", "random_grid", "rule_words"]
