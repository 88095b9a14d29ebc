"""Evaluation features on the HIP path: ROCKET (reference evaluation/rocket_functions.py).
FID / IS / the supervised FCN feature extractor are evaluation outside the hot path."""
from .rocket_functions import (DeviceKernels, apply_kernel, apply_kernels, apply_kernels_device,
                               generate_kernels)

__all__ = ["DeviceKernels", "apply_kernel", "apply_kernels", "apply_kernels_device",
           "generate_kernels"]
