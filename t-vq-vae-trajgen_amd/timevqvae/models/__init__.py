"""Model modules with the reference's names and state_dict keys, run on the HIP kernels.
FCNBaseline (the evaluation feature extractor) is not on the hot path."""
from .vq import VectorQuantize
from .vq_vae import VQVAEDecoder, VQVAEEncoder
from .bidirectional_transformer import BidirectionalTransformer
from .maskgit import MaskGIT
from .fidelity_enhancer import FidelityEnhancer, Unet1D

__all__ = ["VectorQuantize", "VQVAEEncoder", "VQVAEDecoder", "BidirectionalTransformer", "MaskGIT", "FidelityEnhancer", "Unet1D"]
