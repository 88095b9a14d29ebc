"""ctypes binding of libtvq_hip.so (include/tvq.h).

The library is loaded after `import torch` so that its NEEDED libamdhip64.so.7
resolves to the HIP runtime torch already mapped (same soname): the kernels
share torch's device context and streams.  There is no fallback: if the
library is missing or no GPU is present, the first call raises.
"""
import ctypes
import os
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get(
    "TVQ_HIP_LIB", os.path.join(os.path.dirname(os.path.dirname(_HERE)), "lib", "libtvq_hip.so"))

P = ctypes.c_void_p
I64 = ctypes.c_int64
I32 = ctypes.c_int
F32 = ctypes.c_float

# name -> argtypes (stream last).  Kept in sync with include/tvq.h (a CPU test
# checks every declared symbol is exported and listed here).
SIGNATURES = {}
_lib = None
_lock = threading.Lock()


def sig(name, *argtypes, restype=I32):
    SIGNATURES[name] = (list(argtypes), restype)


# --- VQ codebook -----------------------------------------------------------
sig("tvq_vq_sqnorm", P, I64, I64, P, P)
sig("tvq_vq_assign_nblocks", I64, restype=I64)
sig("tvq_vq_assign", P, I64, I64, I64, I64, I64, I64, P, P, I64, I32, P, P, P, P, P)
sig("tvq_vq_stats", P, I64, I64, I64, I64, I64, I64, P, I64, P, P, P, P)
sig("tvq_vq_ema", P, P, I64, I64, F32, P, P, P)
sig("tvq_vq_finalize", P, P, I64, I64, F32, P, P, I64, P, P, I64, P, P)
sig("tvq_vq_backward", P, P, P, P, I64, I64, P, P)


class NativeError(RuntimeError):
    pass


def lib():
    """Load libtvq_hip.so once; raise loudly if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise NativeError(
                f"libtvq_hip.so not found at {LIB_PATH}; build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")
        h = ctypes.CDLL(LIB_PATH)
        h.tvq_last_error.restype = ctypes.c_char_p
        h.tvq_last_error.argtypes = []
        h.tvq_abi_version.restype = I32
        for name, (args, res) in SIGNATURES.items():
            fn = getattr(h, name)
            fn.argtypes = args
            fn.restype = res
        _lib = h
    return _lib


def stream_ptr():
    return torch.cuda.current_stream().cuda_stream


def ptr(t):
    """Device pointer of a tensor (None -> NULL).  Rejects CPU tensors loudly."""
    if t is None:
        return None
    if not t.is_cuda:
        raise NativeError("tvq HIP kernels need device tensors (got a CPU tensor); "
                          "the product path has no CPU fallback")
    return t.data_ptr()


def call(name, *args):
    """Call an int-returning entry point; raise with tvq_last_error() on failure."""
    h = lib()
    rc = getattr(h, name)(*args)
    if rc != 0:
        raise NativeError(f"{name} failed ({rc}): {h.tvq_last_error().decode()}")
    return rc


def value(name, *args):
    return getattr(lib(), name)(*args)
