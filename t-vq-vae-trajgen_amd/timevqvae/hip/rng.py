"""Device-resident dropout seed.

Kernels key their dropout masks on (*seed, offset, element index).  The seed lives
in device memory and is advanced once per training step (`advance`), so a
captured hipGraph draws fresh masks on every replay; `offset` = call site + the
call's index since the last `advance`, so an eager step and a graph replay of it draw
identical masks, and repeated calls of one site within a step differ.
"""
import contextlib
import threading

import torch

_seeds = {}
_lock = threading.Lock()
_site = [0]
_calls = [0]
_initial = [0x5EED]


def new_site() -> int:
    """An id for one dropout call site (module), in construction order."""
    _site[0] += 1
    return _site[0] << 40


def call_offset(site: int) -> int:
    _calls[0] += 1
    return (site + _calls[0]) & 0xFFFFFFFFFFFFFFFF


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
    """Seed the dropout stream and restart site numbering, so a model constructed after
    this call draws the same masks as any other model constructed the same way."""
    _initial[0] = int(seed)
    _site[0] = 0
    _calls[0] = 0
    for t in _seeds.values():
        t.fill_(int(seed))


def restart_calls():
    """Restart the per-step call index only (host state; advance() does it too): for a step
    captured in several graphs whose seed advance runs outside them."""
    _calls[0] = 0


def advance(device):
    """Advance the device seed (call once per training step; capturable) and restart the
    per-step call index."""
    _calls[0] = 0
    from ._native import call, ptr, stream_ptr
    call("tvq_add_i64", ptr(seed_tensor(device)), 1, stream_ptr())


_device_decisions = [False]


@contextlib.contextmanager
def device_decisions():
    """Inside the scope, per-step random *control-flow* choices (x-transformers layer
    dropout) are drawn on the device instead of on the host, so a captured graph
    re-draws them on every replay instead of baking in the capture-time choice."""
    prev = _device_decisions[0]
    _device_decisions[0] = True
    try:
        yield
    finally:
        _device_decisions[0] = prev


def decisions_on_device() -> bool:
    return _device_decisions[0]
