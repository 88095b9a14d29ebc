from .vq import VectorQuantize
from .vq_vae import VQVAEDecoder, VQVAEEncoder
from .bidirectional_transformer import BidirectionalTransformer
from .maskgit import MaskGIT

__all__ = ["VectorQuantize", "VQVAEEncoder", "VQVAEDecoder", "BidirectionalTransformer", "MaskGIT"]
