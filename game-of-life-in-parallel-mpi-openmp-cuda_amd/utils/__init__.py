"""I/O, metrics, termination semantics and checkpointing."""
from .termination import reported_generations, sim_phase_at

__all__ = ["reported_generations", "sim_phase_at"]
