"""HIP (gfx950) op layer: ctypes binding of libtvq_hip.so + autograd wrappers."""
from ._native import LIB_PATH, NativeError, lib  # noqa: F401
