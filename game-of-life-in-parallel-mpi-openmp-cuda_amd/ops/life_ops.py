"""Kernel-level ops and independent oracles.

``life_step``       - n generations of the native kernels (HIP or CPU
                      backend) on one periodic grid, no termination logic.
``life_step_torch`` - plain PyTorch fp32 reference: 3x3 ``conv2d`` with
                      circular padding (the oracle SURVEY 4.3 T1 prescribes;
                      runs on CPU or on the GPU).
``life_step_numpy`` - NumPy ``roll``-sum reference.
"""
from __future__ import annotations

import numpy as np

from .._native import native


def life_step(grid: np.ndarray, gens: int = 1, engine: str = "auto", layout: str = "auto",
              tmax: int = 0, epoch: int = 0, device: int = 0) -> np.ndarray:
    """Advance ``grid`` (H x W, 0/1 uint8) by exactly ``gens`` generations."""
    from ..models.life import LifeConfig, Simulation  # noqa: PLC0415

    g = np.ascontiguousarray(grid, dtype=np.uint8)
    H, W = g.shape
    cfg = LifeConfig(W, H, gen_limit=int(gens), layout=layout, tmax=tmax, epoch=epoch)
    sim = Simulation(cfg, engine=engine, device=device)
    sim.load(g)
    sim.advance(int(gens))
    return sim.tile()


def life_step_numpy(grid: np.ndarray, gens: int = 1) -> np.ndarray:
    g = (np.asarray(grid) != 0).astype(np.uint8)
    for _ in range(gens):
        n = sum(np.roll(np.roll(g, dy, 0), dx, 1) for dy in (-1, 0, 1) for dx in (-1, 0, 1)
                if (dy, dx) != (0, 0))
        g = ((n == 3) | ((n == 2) & (g == 1))).astype(np.uint8)
    return g


def life_step_torch(grid, gens: int = 1, device: str = "cpu"):
    """fp32 PyTorch reference of B3/S23 on a torus (conv2d, circular pad)."""
    import torch  # noqa: PLC0415
    import torch.nn.functional as F  # noqa: PLC0415

    t = torch.as_tensor(np.asarray(grid) != 0, dtype=torch.float32, device=device)[None, None]
    k = torch.ones(1, 1, 3, 3, dtype=torch.float32, device=device)
    k[0, 0, 1, 1] = 0.0
    for _ in range(gens):
        n = F.conv2d(F.pad(t, (1, 1, 1, 1), mode="circular"), k)
        t = ((n == 3) | ((n == 2) & (t == 1))).to(torch.float32)
    return t[0, 0].to(torch.uint8).cpu().numpy()


def life_step_torch_roll(grid, gens: int = 1, device: str = "cpu"):
    """fp32 PyTorch reference of B3/S23 on a torus from elementwise ops only
    (separable neighbour sums of rolled copies, no convolution library): the
    verification oracle for whole-benchmark grids, where a first conv2d call
    spends a minute in kernel selection on a fresh box."""
    import torch  # noqa: PLC0415

    t = torch.as_tensor(np.asarray(grid) != 0, dtype=torch.float32, device=device)
    for _ in range(gens):
        h = t + torch.roll(t, 1, 1) + torch.roll(t, -1, 1)
        n = h + torch.roll(h, 1, 0) + torch.roll(h, -1, 0) - t
        t = ((n == 3) | ((n == 2) & (t == 1))).to(torch.float32)
        del h, n
    return t.to(torch.uint8).cpu().numpy()


def random_grid(width: int, height: int, seed: int = 1, density: float = 0.5) -> np.ndarray:
    """Host copy of the engine's counter-based RNG grid (same as init_random)."""
    return native().random_grid(int(width), int(height), int(seed), float(density))


def rule_words(*words: int) -> int:
    """Host emulation of the bit-sliced rule on one word (for ISA-level tests)."""
    return int(native().rule_words(*[int(w) & 0xFFFFFFFF for w in words]))
