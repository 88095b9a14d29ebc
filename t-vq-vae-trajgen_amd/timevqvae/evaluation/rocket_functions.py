"""ROCKET random-convolution features — the reference's evaluation/rocket_functions.py API
(generate_kernels, apply_kernel, apply_kernels; :21-126) with the transform on the GPU.

The reference runs `apply_kernels` with numba on the host cores for every FID/IS feature
extraction (sampler.py:184-189, metrics.py:116-119).  Here the kernels' parameters stay
host numpy arrays (same tuple layout), and the transform is `tvq_rocket_apply`
(csrc/tvq_rocket.hip): float64, unfused multiply/add in the reference's order, so the
features equal the reference's interpreted float64 loop bit for bit.  `apply_kernels`
takes and returns numpy like the reference; `apply_kernels_device` keeps CUDA tensors on
the device.  There is no CPU fallback.
"""
import numpy as np
import torch

from ..hip._native import call, ptr, stream_ptr

MAX_KERNEL_LENGTH = 16


def generate_kernels(input_length, num_kernels):
    """rocket_functions.py:21-57: lengths from {7, 9, 11}, mean-centred N(0,1) weights,
    U(-1,1) biases, dilation 2**U(0, log2((L-1)/(len-1))) truncated, padding half the
    dilated span with probability 1/2.  Draws from numpy's global RNG in the reference's
    order (the reference's numba build draws the same distribution from numba's stream)."""
    candidate_lengths = np.array((7, 9, 11), dtype=np.int32)
    lengths = np.random.choice(candidate_lengths, num_kernels).astype(np.int32)
    weights = np.zeros(lengths.sum(), dtype=np.float64)
    biases = np.zeros(num_kernels, dtype=np.float64)
    dilations = np.zeros(num_kernels, dtype=np.int32)
    paddings = np.zeros(num_kernels, dtype=np.int32)
    a1 = 0
    for i in range(num_kernels):
        n = int(lengths[i])
        w = np.random.normal(0, 1, n)
        weights[a1:a1 + n] = w - w.mean()
        biases[i] = np.random.uniform(-1, 1)
        dilation = np.int32(2 ** np.random.uniform(0, np.log2((input_length - 1) / (n - 1))))
        dilations[i] = dilation
        paddings[i] = ((n - 1) * dilation) // 2 if np.random.randint(2) == 1 else 0
        a1 += n
    return weights, lengths, biases, dilations, paddings


class DeviceKernels:
    """The kernel tuple resident on one device (+ per-kernel weight offsets)."""

    def __init__(self, kernels, device):
        weights, lengths, biases, dilations, paddings = kernels
        lengths = np.asarray(lengths, dtype=np.int32)
        if len(lengths) == 0:
            raise ValueError("rocket: no kernels")
        if lengths.min() < 1 or lengths.max() > MAX_KERNEL_LENGTH:
            raise ValueError(f"rocket: kernel lengths must be in 1..{MAX_KERNEL_LENGTH}")
        if np.asarray(dilations).min() < 1:
            raise ValueError("rocket: dilations must be >= 1")
        woff = np.zeros(len(lengths), dtype=np.int32)
        woff[1:] = np.cumsum(lengths)[:-1]
        if int(lengths.sum()) != len(weights):
            raise ValueError("rocket: weights do not match the kernel lengths")

        def t(a, dt):
            return torch.as_tensor(np.ascontiguousarray(a), dtype=dt).to(device)
        self.weights = t(weights, torch.float64)
        self.woff = t(woff, torch.int32)
        self.lengths = t(lengths, torch.int32)
        self.biases = t(biases, torch.float64)
        self.dilations = t(dilations, torch.int32)
        self.paddings = t(paddings, torch.int32)
        self.num_kernels = len(lengths)
        self.device = torch.device(device)


def apply_kernels_device(X, dk):
    """X (n, L) float64 CUDA tensor, dk: DeviceKernels -> (n, 2 * num_kernels) float64 CUDA
    tensor [ppv, max] per kernel (rocket_functions.py:91-126)."""
    if X.dim() != 2 or X.dtype != torch.float64:
        raise ValueError("rocket: X must be a (n, L) float64 tensor")
    if X.stride(1) != 1:
        X = X.contiguous()
    n, L = X.shape
    out = torch.empty((n, 2 * dk.num_kernels), device=X.device, dtype=torch.float64)
    ldx = X.stride(0) if n > 1 else L  # a size-1 dim may carry any stride (numpy gives 0)
    call("tvq_rocket_apply", ptr(X), n, L, ldx, ptr(dk.weights), ptr(dk.woff),
         ptr(dk.lengths), ptr(dk.biases), ptr(dk.dilations), ptr(dk.paddings), dk.num_kernels,
         ptr(out), stream_ptr())
    return out


def apply_kernels(X, kernels, device=None):
    """rocket_functions.py:91-126: X (n, L) -> (n, 2 * num_kernels) float64 numpy."""
    device = torch.device(device) if device is not None else torch.device(
        "cuda", torch.cuda.current_device())
    dk = kernels if isinstance(kernels, DeviceKernels) else DeviceKernels(kernels, device)
    Xt = torch.as_tensor(np.ascontiguousarray(X, dtype=np.float64)).to(dk.device)
    return apply_kernels_device(Xt, dk).cpu().numpy()


def apply_kernel(X, weights, length, bias, dilation, padding):
    """rocket_functions.py:60-88: one series, one kernel -> (ppv, max)."""
    k = (np.asarray(weights, np.float64), np.array([length], np.int32),
         np.array([bias], np.float64), np.array([dilation], np.int32),
         np.array([padding], np.int32))
    f = apply_kernels(np.asarray(X, np.float64)[None, :], k)[0]
    return float(f[0]), float(f[1])
