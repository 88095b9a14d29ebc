"""timevqvae — MI355X-native TimeVQVAE hot path.

Drop-in for the reference package's hot-path API (SynthAIr/T-VQ-VAE-TrajGen,
timevqvae.models.{vq,vq_vae,maskgit,bidirectional_transformer} and the
timevqvae.utils helpers they use).  Compute runs in libtvq_hip.so (HIP, gfx950)
through the ctypes layer in timevqvae.hip; there is no CPU fallback.
"""
__version__ = "0.1.0"
