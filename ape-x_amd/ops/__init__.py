"""Native extension loader.

``cpu()``  -> ``_apex_cpu`` (host C++ replay core; always available, auto-built).
``hip()``  -> ``_apex_hip`` (gfx950 HIP kernels).  On a machine with a GPU this
raises if the extension is missing or fails to load: there is deliberately no silent
PyTorch fallback for the engine's hot ops.
"""
from __future__ import annotations

import importlib
import importlib.util
import os
import sys
import threading

_lock = threading.Lock()
_mods: dict[str, object] = {}
_HERE = os.path.dirname(os.path.abspath(__file__))


def _load(name: str, builder):
    with _lock:
        if name in _mods:
            return _mods[name]
        if _HERE not in sys.path:
            sys.path.insert(0, _HERE)
        try:
            mod = importlib.import_module(name)
        except ImportError:
            if os.environ.get("APEX_NO_AUTOBUILD") == "1":
                raise
            builder()
            importlib.invalidate_caches()
            mod = importlib.import_module(name)
        _mods[name] = mod
        return mod


def cpu():
    """``APEX_CPU_EXT_DIR`` loads the module from another directory instead (the
    ASan/UBSan build of the sanitizer test, ``build.build_cpu(sanitize=True)``)."""
    from . import build

    alt = os.environ.get("APEX_CPU_EXT_DIR")
    if alt:
        with _lock:
            if "_apex_cpu" not in _mods:
                spec = importlib.util.spec_from_file_location("_apex_cpu", os.path.join(alt, build.cpu_target().name))
                mod = importlib.util.module_from_spec(spec)
                spec.loader.exec_module(mod)
                _mods["_apex_cpu"] = mod
            return _mods["_apex_cpu"]
    return _load("_apex_cpu", lambda: build.build_cpu())


def hip():
    """Load the gfx950 kernel library (requires ``import torch`` first, done here).
    ``APEX_HIP_EXT_DIR`` loads it from another directory instead (whole-step A/B of two
    builds in separate processes on one box: ``scripts/ab/apex_engine_ab.py``)."""
    import torch  # noqa: F401  -- binds libamdhip64.so.7 to torch's copy before our dlopen
    from . import build

    alt = os.environ.get("APEX_HIP_EXT_DIR")
    if alt:
        with _lock:
            if "_apex_hip" not in _mods:
                spec = importlib.util.spec_from_file_location("_apex_hip", os.path.join(alt, build.hip_target().name))
                mod = importlib.util.module_from_spec(spec)
                spec.loader.exec_module(mod)
                _mods["_apex_hip"] = mod
            return _mods["_apex_hip"]
    return _load("_apex_hip", lambda: build.build_hip())


def hip_available() -> bool:
    try:
        import torch

        if not torch.cuda.is_available():
            return False
        hip()
        return True
    except Exception:
        return False


def native_paths() -> list[str]:
    return [getattr(m, "__file__", "?") for m in _mods.values()]
