"""Utilities with the reference ``utils`` surface (utils.py:9-97) plus metrics,
timing and checkpoint helpers.

``compute_loss`` / ``compute_loss_AQL`` / ``update_parameters`` are re-exported from
:mod:`apex_amd.algo` so ``from apex_amd import utils; utils.compute_loss(...)``
works like the reference module.
"""
from __future__ import annotations

import io
import random

import numpy as np

from ..algo.losses import compute_loss, compute_loss_AQL, update_parameters  # noqa: F401
from .tb import NullWriter, SummaryWriter  # noqa: F401


def print_args(args):
    print(" " * 26 + "Options")
    for k, v in vars(args).items():
        print(" " * 26 + k + ": " + str(v))


def set_global_seeds(seed, use_torch=False):
    if use_torch:
        import torch

        torch.manual_seed(seed)
        if torch.cuda.is_available():
            torch.cuda.manual_seed(seed)
    np.random.seed(seed)
    random.seed(seed)


def array2png(arr):
    from PIL import Image

    img = Image.fromarray(arr)
    buf = io.BytesIO()
    img.save(buf, format="PNG")
    out = buf.getvalue()
    buf.close()
    img.close()
    return out


def png2array(png):
    from PIL import Image

    buf = io.BytesIO(png)
    img = Image.open(buf)
    arr = np.array(img)
    img.close()
    buf.close()
    return arr
