"""Device-resident dropout seed.

Kernels key their dropout masks on (*seed, offset, element index).  The seed lives
in device memory and is advanced once per training step (`advance`), so a
captured hipGraph draws fresh masks on every replay; `offset` separates call
sites (and eager calls) on the host side.
"""
import itertools
import threading

import torch

_seeds = {}
_lock = threading.Lock()
_site = itertools.count(1)
_calls = itertools.count(1)
_initial = [0x5EED]


def new_site() -> int:
    """A unique id for one dropout call site (module)."""
    return next(_site) << 40


def call_offset(site: int) -> int:
    return (site + next(_calls)) & 0xFFFFFFFFFFFFFFFF


def seed_tensor(device) -> torch.Tensor:
    device = torch.device(device)
    key = (device.type, device.index if device.index is not None else torch.cuda.current_device())
    t = _seeds.get(key)
    if t is None:
        with _lock:
            t = _seeds.get(key)
            if t is None:
                t = torch.full((1,), _initial[0], dtype=torch.int64, device=device)
                _seeds[key] = t
    return t


def manual_seed(seed: int):
    _initial[0] = int(seed)
    for t in _seeds.values():
        t.fill_(int(seed))


def advance(device):
    """Advance the device seed (call once per training step; capturable)."""
    seed_tensor(device).add_(1)
