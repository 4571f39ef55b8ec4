"""The reference's termination semantics as a pure function.

Serial loop (src/game.c:169-196): at generation t (1-based) it first stops if
G_{t-1} is empty (reports t-1), evolves G_t, and every SIMILARITY_FREQUENCY-th
iteration stops if G_t == G_{t-1} (reports t-1, because the break skips
``generation++``).  Both conditions are absorbing, so everything follows from
g_f = the first generation with G_{g_f} == G_{g_f-1}:

* if the grid at g_f is empty, the run died at g_f - 1 -> reports g_f - 1;
* else the first similarity check t >= g_f reports t - 1 (if t <= limit);
* else the run reaches the limit.

The native engine implements the same rule (csrc/src/engine.cpp); this
mirror is used for chunked/checkpointed runs and as a test oracle.
"""
from __future__ import annotations


def reported_generations(first_unchanged: int, extinct: bool, limit: int, start_gen: int = 0,
                         check_similarity: bool = True, sim_freq: int = 3,
                         sim_phase: int = 0) -> tuple[int, str]:
    """Return (Generations value, stop reason) for a run over (start_gen, limit]."""
    if first_unchanged < 0 or first_unchanged > limit:
        return limit, "limit"
    if extinct:
        return first_unchanged - 1, "extinction"
    if check_similarity:
        k = first_unchanged - start_gen + sim_phase
        tsim = first_unchanged + ((sim_freq - (k % sim_freq)) % sim_freq)
        if tsim <= limit:
            return tsim - 1, "similarity"
    return limit, "fixed_point"


def sim_phase_at(gen: int, start_gen: int = 0, sim_phase: int = 0, sim_freq: int = 3) -> int:
    """Similarity counter value after generation ``gen`` (no check fired)."""
    return (gen - start_gen + sim_phase) % sim_freq
