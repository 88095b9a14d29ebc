"""Evaluation features on the HIP path: ROCKET (reference evaluation/rocket_functions.py)
and FID / IS (reference evaluation/eval_utils.py; the FID moments on the device).  The
supervised FCN feature extractor is evaluation outside the hot path."""
from .eval_utils import calculate_fid, calculate_inception_score, feature_moments
from .rocket_functions import (DeviceKernels, apply_kernel, apply_kernels, apply_kernels_device,
                               generate_kernels)

__all__ = ["DeviceKernels", "apply_kernel", "apply_kernels", "apply_kernels_device",
           "calculate_fid", "calculate_inception_score", "feature_moments", "generate_kernels"]
