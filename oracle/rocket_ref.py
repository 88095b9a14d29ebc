"""TEST INFRASTRUCTURE ONLY — numpy wrapper over oracle/build/librocket_ref.so (rocket_ref.c),
the C restatement of evaluation/rocket_functions.py:60-126 (apply_kernel / apply_kernels)."""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "build", "librocket_ref.so")
_lib = None


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            subprocess.check_call(["make", "-s", "-C", _HERE])
        _lib = ctypes.CDLL(_SO)
        P, L, I = ctypes.c_void_p, ctypes.c_long, ctypes.c_int
        _lib.rocketref_apply.argtypes = [P, L, L, L, P, P, P, P, P, L, P, I]
        _lib.rocketref_apply.restype = None
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def apply_kernels(X, kernels, threads=1):
    """X (n, L) float64, kernels = (weights, lengths, biases, dilations, paddings) as
    generate_kernels returns them -> (n, 2 * num_kernels) float64 [ppv, max] per kernel."""
    X = np.ascontiguousarray(X, dtype=np.float64)
    w, lengths, biases, dil, pad = kernels
    w = np.ascontiguousarray(w, dtype=np.float64)
    lengths = np.ascontiguousarray(lengths, dtype=np.int32)
    biases = np.ascontiguousarray(biases, dtype=np.float64)
    dil = np.ascontiguousarray(dil, dtype=np.int32)
    pad = np.ascontiguousarray(pad, dtype=np.int32)
    n, L = X.shape
    nk = len(lengths)
    out = np.empty((n, 2 * nk), np.float64)
    _load().rocketref_apply(_p(X), n, L, L, _p(w), _p(lengths), _p(biases), _p(dil), _p(pad),
                            nk, _p(out), int(threads))
    return out
