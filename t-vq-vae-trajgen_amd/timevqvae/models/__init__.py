from .vq import VectorQuantize
from .vq_vae import VQVAEDecoder, VQVAEEncoder
from .bidirectional_transformer import BidirectionalTransformer
from .maskgit import MaskGIT
from .fidelity_enhancer import FidelityEnhancer, Unet1D

__all__ = ["VectorQuantize", "VQVAEEncoder", "VQVAEDecoder", "BidirectionalTransformer", "MaskGIT", "FidelityEnhancer", "Unet1D"]
