"""Model family: B3/S23 Life on a periodic torus (the reference's only model)."""
from .life import LifeConfig, RunReport, Simulation, make_backend, reference_run, simulate

__all__ = ["LifeConfig", "RunReport", "Simulation", "make_backend", "reference_run", "simulate"]
