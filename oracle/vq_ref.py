"""TEST INFRASTRUCTURE ONLY — numpy wrapper over oracle/build/libvq_ref.so (vq_ref.c)."""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "build", "libvq_ref.so")
_lib = None


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            subprocess.check_call(["make", "-s", "-C", _HERE])
        _lib = ctypes.CDLL(_SO)
        P, L, F = ctypes.c_void_p, ctypes.c_long, ctypes.c_float
        _lib.vqref_assign.argtypes = [P, L, L, P, L, P, P, P]
        _lib.vqref_assign.restype = None
        _lib.vqref_ema.argtypes = [P, P, L, L, L, F, F, P, P, P, P, P]
        _lib.vqref_ema.restype = None
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def assign(x, E):
    """x (M,D) f32, E (K,D) f32 -> (idx int64 (M,), best dist f32 (M,), fp64 top-2 gap (M,))."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    E = np.ascontiguousarray(E, dtype=np.float32)
    M, D = x.shape
    K = E.shape[0]
    idx = np.empty(M, np.int64)
    best = np.empty(M, np.float32)
    gap = np.empty(M, np.float64)
    _load().vqref_assign(_p(x), M, D, _p(E), K, _p(idx), _p(best), _p(gap))
    return idx, best, gap


def ema(x, idx, cluster_size, embed_avg, decay=0.8, eps=1e-5):
    """Returns (cluster_size', embed_avg', embed', counts, perplexity) (vq.py:227-247)."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    idx = np.ascontiguousarray(idx, dtype=np.int64)
    cs = np.array(cluster_size, dtype=np.float32, copy=True)
    ea = np.array(embed_avg, dtype=np.float32, copy=True)
    K, D = ea.shape
    E = np.empty_like(ea)
    counts = np.empty(K, np.float32)
    perp = np.empty(1, np.float32)
    _load().vqref_ema(_p(x), _p(idx), x.shape[0], D, K, decay, eps, _p(cs), _p(ea), _p(E),
                      _p(counts), _p(perp))
    return cs, ea, E, counts, float(perp[0])
