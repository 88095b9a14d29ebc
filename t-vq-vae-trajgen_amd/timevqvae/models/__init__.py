from .vq import VectorQuantize
from .vq_vae import VQVAEDecoder, VQVAEEncoder

__all__ = ["VectorQuantize", "VQVAEEncoder", "VQVAEDecoder"]
