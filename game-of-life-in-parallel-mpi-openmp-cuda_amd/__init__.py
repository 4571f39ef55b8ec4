"""gol-mi355x: an MI355X-native Game of Life stencil engine.

Same capabilities as v-pap/Game-of-Life-in-parallel-MPI-OpenMP-CUDA (serial,
MPI with three I/O strategies, MPI+OpenMP and CUDA programs evolving B3/S23 on
a torus), rebuilt as one engine: CDNA4 HIP kernels (bit-sliced, temporal
blocking in registers), a C++ runtime (epochs, deep halos, lazy exact
termination, parallel text I/O) and RCCL halos over xGMI with one process
per GPU.

Import as ``gol_amd`` (symlink to this directory).
"""
from ._native import hip_available, native
from .models.life import LifeConfig, RunReport, Simulation, make_backend, reference_run, simulate
from .ops.life_ops import life_step, life_step_numpy, life_step_torch, random_grid

__version__ = "0.1.0"

__all__ = ["LifeConfig", "RunReport", "Simulation", "make_backend", "reference_run", "simulate",
           "life_step", "life_step_numpy", "life_step_torch", "random_grid", "native",
           "hip_available", "__version__"]
