"""Sampling from trained models (reference generation/): the sampling half of TrainedModelSampler."""
from .sampler import TrainedModelSampler

__all__ = ["TrainedModelSampler"]
