"""Device and RNG defaults for model construction.

Models are created on the current HIP device.  On a host without a GPU the
parameters are created on the CPU so that configuration and host logic can be
inspected, but every compute call then fails loudly in hip_ops (libtt has no
CPU path).
"""
from __future__ import annotations

from typing import Optional

import torch

_seed: Optional[int] = None


def set_seed(seed: Optional[int]) -> None:
    """Seed for parameter initialisation (None = torch's default RNG state)."""
    global _seed
    _seed = seed


def make_generator(seed: Optional[int] = None) -> torch.Generator:
    g = torch.Generator(device="cpu")
    s = seed if seed is not None else _seed
    if s is not None:
        g.manual_seed(int(s))
    else:
        g.seed()
    return g


def default_device() -> torch.device:
    if torch.cuda.is_available():
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")
