"""Loader for the in-tree native library ``_pz_C.so`` (HIP kernels + host C++ runtime).

The library registers the ``torch.ops.pz`` namespace (see ``csrc/bindings.cpp``). It is built
in-tree by :mod:`penr_oz_neural_network_torch_amd._build` (``hipcc --offload-arch=gfx950``) so
the ``.so`` travels with the repository snapshot to the GPU box.

Policy:

* On a machine **with** a GPU, a missing or unloadable library is an error the moment a GPU op
  is requested (:func:`require`): GPU code never silently falls back to ATen.
* On a CPU-only machine, host-side helpers (e.g. the JSON array formatter) fall back to their
  pure-Python equivalents, which produce identical results.
"""
from __future__ import annotations

import os
import threading

import torch

_PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_NAME = "_pz_C.so"
_lock = threading.Lock()
_state: dict = {"loaded": False, "error": None, "path": None}


def library_path() -> str:
    return os.path.join(_PKG_DIR, LIB_NAME)


def load(raise_on_error: bool = False) -> bool:
    """Load the library once; returns True when ``torch.ops.pz`` is available."""
    with _lock:
        if _state["loaded"]:
            return True
        path = library_path()
        if not os.path.exists(path):
            _state["error"] = f"{path} not built (run `python -m penr_oz_neural_network_torch_amd._build`)"
        else:
            try:
                torch.ops.load_library(path)
                _state["loaded"] = True
                _state["path"] = path
                _state["error"] = None
            except Exception as e:  # pragma: no cover - depends on the box
                _state["error"] = f"failed to load {path}: {e}"
        if not _state["loaded"] and raise_on_error:
            raise RuntimeError(_state["error"])
        return _state["loaded"]


def require() -> None:
    """Fail loudly if the native library is unavailable (used by every GPU op)."""
    load(raise_on_error=True)


def has_host_ops() -> bool:
    return load()


def error() -> str | None:
    return _state["error"]


def format_json_array(t: torch.Tensor, level: int) -> str:
    return torch.ops.pz.format_json_array(t, level)


def built_sources_stale() -> bool:
    """True when the built library does not match the current csrc/ content (the build's
    content-hash manifest, ``_build.is_fresh``; dev helper)."""
    from .. import _build
    return not _build.is_fresh()
