"""Hot-path subset of the reference timevqvae/utils/train_utils.py (same names and
signatures).  Arithmetic runs in libtvq_hip.so; host-only helpers (schedulers,
YAML, seeding) are plain Python."""
import random
from typing import Union

import numpy as np
import torch
import torch.nn as nn
import yaml
from torch.optim.lr_scheduler import CosineAnnealingLR, LambdaLR, SequentialLR

from ..hip import signal as _sig
from ..hip.norm import snake as _snake


def load_yaml_param_settings(yaml_fname: str):
    """train_utils.py:86-92 (SafeLoader: the configs are plain YAML)."""
    with open(yaml_fname, "r") as f:
        return yaml.safe_load(f)


def set_seed(seed: int) -> None:
    """train_utils.py:44-59."""
    torch.manual_seed(seed)
    np.random.seed(seed)
    random.seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)
    from ..hip import rng
    rng.manual_seed(seed)


def freeze(model):
    """train_utils.py:250-252."""
    for p in model.parameters():
        p.requires_grad = False


def unfreeze(model):
    """train_utils.py:255-257."""
    for p in model.parameters():
        p.requires_grad = True


def time_to_timefreq(x, n_fft: int, C: int, norm: bool = True):
    """train_utils.py:293-307: (B,C,L) -> (B,2C,3,L+1), channel = 2c + {real, imag}."""
    if n_fft != 4 or not norm:
        raise NotImplementedError("the HIP STFT implements n_fft=4, normalized=True (config.yaml)")
    return _sig.stft_encode(x, raw=True)["raw"]


def timefreq_to_time(x, n_fft: int, C: int, norm: bool = True):
    """train_utils.py:310-321: (B,2C,3,W) -> (B,C,W-1)."""
    if n_fft != 4 or not norm:
        raise NotImplementedError("the HIP iSTFT implements n_fft=4, normalized=True (config.yaml)")
    return _sig.istft_decode(x, C, "all", x.shape[-1] - 1)


def quantize(z, vq_model, transpose_channel_length_axes=False, svq_temp: Union[float, None] = None):
    """train_utils.py:338-358.  The 'b c h w -> b (h w) c' rearrange is a VIEW; the VQ
    kernels read and write it with strides (no transpose is materialised)."""
    input_dim = len(z.shape) - 2
    if input_dim == 2:
        b, c, h, w = z.shape
        zt = z.flatten(2).transpose(1, 2)
        z_q, indices, vq_loss, perplexity = vq_model(zt, svq_temp)
        z_q = z_q.transpose(1, 2).reshape(b, c, h, w)
    elif input_dim == 1:
        if transpose_channel_length_axes:
            z = z.transpose(1, 2)
        z_q, indices, vq_loss, perplexity = vq_model(z, svq_temp)
        if transpose_channel_length_axes:
            z_q = z_q.transpose(1, 2)
    else:
        raise ValueError
    return z_q, indices, vq_loss, perplexity


def zero_pad_high_freq(xf, copy=False):
    """train_utils.py:361-372 (keep the LF bin).  Plain data movement; the hot path
    fuses it into the HIP STFT / iSTFT kernels."""
    if not copy:
        out = torch.zeros_like(xf)
        out[:, :, 0, :] = xf[:, :, 0, :]
        return out
    return xf[:, :, :1, :].expand(-1, -1, xf.shape[2], -1).float().contiguous()


def zero_pad_low_freq(xf, copy=False):
    """train_utils.py:375-386 (keep the HF bins)."""
    if not copy:
        out = torch.zeros_like(xf)
        out[:, :, 1:, :] = xf[:, :, 1:, :]
        return out
    return torch.cat((xf[:, :, 1:2, :], xf[:, :, 1:, :]), dim=2).float()


def band_of(pad_func) -> str:
    """'lf' for zero_pad_high_freq, 'hf' for zero_pad_low_freq (the encoder/decoder pad_func)."""
    name = getattr(pad_func, "__name__", "")
    if pad_func is zero_pad_high_freq or name == "zero_pad_high_freq":
        return "lf"
    if pad_func is zero_pad_low_freq or name == "zero_pad_low_freq":
        return "hf"
    raise NotImplementedError(f"pad_func {pad_func!r}: only zero_pad_high_freq/low_freq are fused")


def compute_downsample_rate(input_length: int, n_fft: int, downsampled_width: int):
    """train_utils.py:413-418."""
    return (round(input_length / (np.log2(n_fft) - 1) / downsampled_width)
            if input_length >= downsampled_width else 1)


class SnakeActivation(nn.Module):
    """train_utils.py:421-448: x + (1/a) sin(a x)^2 with per-channel learnable a
    (init U(a_base, a_max) via np.random, as the reference)."""

    def __init__(self, num_features: int, dim: int, a_base=0.2, learnable=True, a_max=0.5):
        super().__init__()
        assert dim in [1, 2], "`dim` supports 1D and 2D inputs."
        shape = (1, num_features, 1) if dim == 1 else (1, num_features, 1, 1)
        if learnable:
            a = np.random.uniform(a_base, a_max, size=shape)
            self.a = nn.Parameter(torch.tensor(a, dtype=torch.float32))
        else:
            self.register_buffer("a", torch.full(shape, a_base, dtype=torch.float32))

    def forward(self, x):
        if self.a.numel() == 1:
            return _snake(x, self.a.reshape(-1).expand(x.shape[1]).contiguous())
        return _snake(x, self.a)


def linear_warmup_cosine_annealingLR(optimizer: torch.optim.Optimizer, max_steps: int,
                                     linear_warmup_rate: float = 0.1, min_lr: float = 1e-6):
    """train_utils.py:451-483 (torch schedulers; host-side)."""
    assert 0.0 < linear_warmup_rate < 1.0, "0 < linear_warmup_rate < 1."
    warmup_steps = int(max_steps * linear_warmup_rate)

    def warmup_lambda(current_step):
        if current_step >= warmup_steps:
            return 1.0
        return float(current_step) / float(max(1, warmup_steps))

    warmup = LambdaLR(optimizer, lr_lambda=warmup_lambda)
    cosine = CosineAnnealingLR(optimizer, max_steps - warmup_steps, eta_min=min_lr)
    return SequentialLR(optimizer, schedulers=[warmup, cosine], milestones=[warmup_steps])


def remove_outliers(data: np.ndarray):
    """train_utils.py:486-493: keep the rows an IsolationForest (max_samples 0.9,
    contamination 0.1, random_state 0) labels inliers -- host sklearn, as the reference."""
    from sklearn.ensemble import IsolationForest
    keep = IsolationForest(max_samples=0.9, contamination=0.1, random_state=0).fit_predict(data) == 1
    return data[keep]
