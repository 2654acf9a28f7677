"""Checkpoints.

Primary artifact: ``torch.save(model.state_dict(), path)`` with the reference keys,
shapes and fp32 dtype, so the reference ``enjoy.py`` / ``load_model`` can read it
(origin_repo/learner.py:166-168, ApeX.py:74-86, DQN.py:117-122).

Sidecar ``<path>.train.pt`` (build addition) makes resume exact instead of
weights-only: target net, optimizer + LR-scheduler state, step counters and the
host RNG states.  Everything is stored as tensors / plain containers, so both files
load with ``torch.load(..., weights_only=True)`` (no pickled code is executed).
"""
from __future__ import annotations

import os
import random

import numpy as np
import torch


def _cpu_state_dict(model) -> dict:
    return {k: v.detach().to("cpu", copy=True).contiguous() for k, v in model.state_dict().items()}


def save_model(model, path: str) -> str:
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    tmp = path + ".tmp"
    torch.save(_cpu_state_dict(model), tmp)
    os.replace(tmp, path)  # atomic: a reader never sees a half-written checkpoint
    return path


def load_model(model, path: str, strict: bool = True):
    sd = torch.load(path, map_location="cpu", weights_only=True)
    model.load_state_dict(sd, strict=strict)
    return model


def sidecar_path(path: str) -> str:
    return path + ".train.pt"


def _rng_state() -> dict:
    py = random.getstate()
    np_state = np.random.get_state()
    return {
        "python_version": int(py[0]), "python_state": torch.tensor(py[1], dtype=torch.int64),
        "python_gauss": -1.0 if py[2] is None else float(py[2]),
        "numpy_keys": torch.from_numpy(np_state[1].astype(np.int64)), "numpy_pos": int(np_state[2]),
        "numpy_has_gauss": int(np_state[3]), "numpy_gauss": float(np_state[4]),
        "torch": torch.get_rng_state(),
    }


def _set_rng_state(st: dict) -> None:
    gauss = None if st["python_gauss"] == -1.0 else st["python_gauss"]
    random.setstate((st["python_version"], tuple(int(x) for x in st["python_state"].tolist()), gauss))
    np.random.set_state(("MT19937", st["numpy_keys"].numpy().astype(np.uint32), st["numpy_pos"],
                         st["numpy_has_gauss"], st["numpy_gauss"]))
    torch.set_rng_state(st["torch"])


def save_train_state(path: str, *, target=None, optimizers=(), schedulers=(), counters: dict | None = None,
                     extra_tensors: dict | None = None) -> str:
    """Write the resume sidecar next to ``path`` (the reference-format model file)."""
    state = {
        "target": _cpu_state_dict(target) if target is not None else {},
        "optimizers": [o.state_dict() for o in optimizers],
        "schedulers": [s.state_dict() for s in schedulers],
        "counters": {k: int(v) for k, v in (counters or {}).items()},
        "rng": _rng_state(),
        "extra": {k: v.detach().cpu() for k, v in (extra_tensors or {}).items()},
    }
    sp = sidecar_path(path)
    tmp = sp + ".tmp"
    torch.save(state, tmp)
    os.replace(tmp, sp)
    return sp


def load_train_state(path: str, *, target=None, optimizers=(), schedulers=(), restore_rng: bool = True) -> dict:
    st = torch.load(sidecar_path(path), map_location="cpu", weights_only=True)
    if target is not None and st["target"]:
        target.load_state_dict(st["target"])
    for o, s in zip(optimizers, st["optimizers"]):
        o.load_state_dict(s)
    for sch, s in zip(schedulers, st["schedulers"]):
        sch.load_state_dict(s)
    if restore_rng:
        _set_rng_state(st["rng"])
    return st
