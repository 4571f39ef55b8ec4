"""Loader for the native extension ``_gol.so`` (C++ runtime + CDNA4 HIP kernels).

PyTorch is imported first on purpose: torch ships its own ``libamdhip64`` /
``librccl`` (soname ``.so.7`` / ``.so.1``); loading torch first makes our
extension bind to the very same HIP runtime and RCCL instead of pulling a
second copy from ``/opt/rocm/lib`` into the process.

The extension is built in-tree (``native_build.py``).  On a GPU box a missing
or stale extension is a hard error - there is no silent Python fallback for
the engine.
"""
from __future__ import annotations

import importlib
import importlib.util
import os
import threading

_lock = threading.Lock()
_mod = None


def _import_torch_first() -> None:
    if os.environ.get("GOL_NO_TORCH") == "1":
        return
    try:
        import torch  # noqa: F401, PLC0415
    except Exception:  # pragma: no cover - torch is part of the image
        pass


def native():
    """Return the loaded ``_gol`` extension module, building it if needed."""
    global _mod
    if _mod is not None:
        return _mod
    with _lock:
        if _mod is not None:
            return _mod
        _import_torch_first()
        from . import native_build  # noqa: PLC0415

        if not native_build.is_built():
            if os.environ.get("GOL_NO_AUTOBUILD") == "1":
                raise ImportError(
                    "gol_amd native extension is missing or stale; run `python -m gol_amd.native_build`")
            # torchrun starts one process per GPU: build once, the others wait
            # on the lock and find the fresh artefacts.
            import fcntl  # noqa: PLC0415

            with open(native_build.MODULE.parent / ".build.lock", "w") as lk:
                fcntl.flock(lk, fcntl.LOCK_EX)
                if not native_build.is_built():
                    native_build.build()
        alt = os.environ.get("GOL_NATIVE_SO")  # experiment builds (scripts/build_alt.py)
        if alt:
            spec = importlib.util.spec_from_file_location(__package__ + "._gol", alt)
            _mod = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(_mod)
            return _mod
        _mod = importlib.import_module(__package__ + "._gol")
        return _mod


def hip_available() -> bool:
    return bool(native().hip_available())
