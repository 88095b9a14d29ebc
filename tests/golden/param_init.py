"""Deterministic per-key parameter rule shared by make_golden.py and the tests.

Instead of committing multi-MB state_dicts, every floating-point entry of a
Stage1 state_dict is overwritten from an RNG seeded by crc32(key) before the
reference runs.  The tests rebuild the same state_dict from the same rule, so
the fixture only needs inputs, outputs and gradients.  Keys follow the
reference's module tree (trainers/stage1.py:34-87), which the product keeps.
"""
import zlib

import numpy as np


def value_for(key: str, shape, seed: int = 0) -> np.ndarray:
    rng = np.random.default_rng(zlib.crc32(key.encode()) + 7919 * seed)
    shape = tuple(shape)
    leaf = key.rsplit(".", 1)[-1]
    if leaf == "a":  # SnakeActivation.a ~ U(0.2, 0.5) (train_utils.py:438-442)
        return rng.uniform(0.2, 0.5, size=shape).astype(np.float32)
    if leaf == "running_var":
        return rng.uniform(0.5, 1.5, size=shape).astype(np.float32)
    if leaf == "running_mean":
        return (0.1 * rng.standard_normal(shape)).astype(np.float32)
    if leaf == "weight" and len(shape) == 1:  # BN gamma
        return (1.0 + 0.1 * rng.standard_normal(shape)).astype(np.float32)
    if leaf == "bias":
        return (0.05 * rng.standard_normal(shape)).astype(np.float32)
    if leaf in ("embed", "embed_avg"):
        return rng.standard_normal(shape).astype(np.float32)
    if leaf == "cluster_size":
        return rng.uniform(0.0, 2.0, size=shape).astype(np.float32)
    if leaf == "weight":
        fan_in = int(np.prod(shape[1:])) if len(shape) > 1 else 1
        return (rng.standard_normal(shape) / np.sqrt(max(fan_in, 1))).astype(np.float32)
    return rng.standard_normal(shape).astype(np.float32)


def fill_state_dict(sd: dict, seed: int = 0) -> dict:
    """Return {key: np.ndarray} for every floating entry of `sd` (a torch state_dict)."""
    out = {}
    for k, v in sd.items():
        if not v.is_floating_point():
            continue
        if k.endswith("initted"):
            continue
        if k.endswith("embed_avg"):
            # embed_avg starts equal to embed in the reference (vq.py:159,165)
            out[k] = value_for(k[: -len("embed_avg")] + "embed", v.shape, seed)
            continue
        out[k] = value_for(k, v.shape, seed)
    return out
