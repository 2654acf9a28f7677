"""Tracing hooks and HIP debug modes.

The reference has no tracing at all (its only instrumentation is the learner's BPS
print, learner.py:171-175).  Here:

* ``range(name)`` / ``mark(name)``: roctx ranges (rocprofiler-sdk roctx, via ctypes) around
  the engine's host-side phases -- actor step, learner step, parameter publish, target
  sync -- so ``rocprofv3 --marker-trace --kernel-trace`` lines kernels up with the
  Ape-X loop.  Off unless ``enable()`` was called (``--profile 1`` / ``APEX_ROCTX=1``);
  disabled ranges cost one bool test.
* ``hip_debug_env(level)``: ``AMD_LOG_LEVEL`` + ``HIP_LAUNCH_BLOCKING`` (+ serialised
  kernel launches) for fault hunting; only effective before the HIP runtime starts, so
  the CLIs apply it before their first ``torch.cuda`` call.
"""
from __future__ import annotations

import contextlib
import ctypes
import os

_lib = None
_enabled = False


def _load():
    global _lib
    if _lib is None:
        # rocprofiler-sdk's roctx first: rocprofv3 --marker-trace records that one (the
        # legacy roctracer libroctx64 is only seen by the old rocprof)
        for name in ("librocprofiler-sdk-roctx.so.1", "/opt/rocm/lib/librocprofiler-sdk-roctx.so.1",
                     "libroctx64.so", "libroctx64.so.4", "/opt/rocm/lib/libroctx64.so"):
            try:
                _lib = ctypes.CDLL(name)
                break
            except OSError:
                continue
        if _lib is not None:
            _lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            _lib.roctxRangePushA.restype = ctypes.c_int
            _lib.roctxRangePop.restype = ctypes.c_int
            _lib.roctxMarkA.argtypes = [ctypes.c_char_p]
    return _lib


def enable(on: bool = True) -> bool:
    """Turn roctx ranges on (returns False when libroctx64 is unavailable)."""
    global _enabled
    _enabled = bool(on) and _load() is not None
    return _enabled


def enabled() -> bool:
    return _enabled


@contextlib.contextmanager
def range(name: str):  # noqa: A001 -- mirrors roctx naming
    if not _enabled:
        yield
        return
    _lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        _lib.roctxRangePop()


def mark(name: str) -> None:
    if _enabled:
        _lib.roctxMarkA(name.encode())


def hip_debug_env(level: int = 3, blocking: bool = True) -> dict:
    """Set the HIP runtime's debug knobs for this process (and children); returns them."""
    env = {"AMD_LOG_LEVEL": str(int(level))}
    if blocking:
        env.update(HIP_LAUNCH_BLOCKING="1", AMD_SERIALIZE_KERNEL="3", AMD_SERIALIZE_COPY="3")
    os.environ.update(env)
    return env


if os.environ.get("APEX_ROCTX") == "1":
    enable(True)
