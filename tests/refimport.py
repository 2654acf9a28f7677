"""Import the read-only reference modules in-process for differential tests.

The reference needs ``gym`` (absent here) and relies on ``np.array(x, copy=False)``
(an error on NumPy 2).  We register a stub ``gym`` module whose ``spaces`` are this
framework's Box/Discrete and import the reference files under private names with a
NumPy shim applied only inside them.  Nothing from the reference is copied into the
framework; tests skip when /root/reference is absent.
"""
from __future__ import annotations

import importlib.util
import os
import sys
import types

import numpy as np

REF = "/root/reference"


def available() -> bool:
    return os.path.isdir(REF) and os.path.exists(os.path.join(REF, "memory.py"))


def _stub_gym():
    if "gym" in sys.modules:
        return
    from apex_amd.envs import spaces
    from apex_amd.envs.core import Env, Wrapper

    gym = types.ModuleType("gym")
    sp = types.ModuleType("gym.spaces")
    sp.Box = spaces.Box
    sp.Discrete = spaces.Discrete
    gym.spaces = sp
    gym.Env = Env
    gym.Wrapper = Wrapper
    sys.modules["gym"] = gym
    sys.modules["gym.spaces"] = sp


class _NumpyShim(types.ModuleType):
    """numpy proxy mapping np.array(x, copy=False) -> np.asarray(x) (NumPy-2 compat)."""

    def __init__(self):
        super().__init__("numpy")

    def __getattr__(self, name):
        return getattr(np, name)

    @staticmethod
    def array(obj, *args, copy=True, **kw):
        if copy is False:
            return np.asarray(obj, *args, **kw)
        return np.array(obj, *args, **kw)


def load(name: str):
    """Load reference ``<name>.py`` (model / memory / utils) as module ``_ref_<name>``."""
    key = f"_ref_{name}"
    if key in sys.modules:
        return sys.modules[key]
    _stub_gym()
    spec = importlib.util.spec_from_file_location(key, os.path.join(REF, f"{name}.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    if hasattr(mod, "np"):
        mod.np = _NumpyShim()
    sys.modules[key] = mod
    return mod
