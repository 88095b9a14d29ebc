from .vq import VectorQuantize

__all__ = ["VectorQuantize"]
