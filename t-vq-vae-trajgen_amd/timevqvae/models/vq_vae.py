"""Stage1 encoder/decoder — same API and module tree as the reference
timevqvae/models/vq_vae.py (state_dict keys `encoder.{i}.block.0.weight`,
`convs.{0..5}`, `proj`, `decoder.{i}`, `linear` ... are identical), executed by
the HIP kernels:

  VQVAEEncBlock  replicate-pad Conv2d(3x4, s(1,2)) -> [BN + Snake fused]
  ResBlock       Snake -> Conv2d(3x3) -> [BN + Snake] -> Conv2d(3x3) with the
                 dropout and the residual (identity or 1x1 proj) fused into the
                 second conv's epilogue
  VQVAEDecBlock  ConvTranspose2d(3x4, s(1,2)) -> [BN + Snake]
  encoder input  one fused STFT + band-copy kernel; decoder tail one fused
                 band-mask + iSTFT + linear-interp kernel, then Linear(T,T) with
                 the residual in the GEMM epilogue.
"""
import numpy as np
import torch
import torch.nn as nn

from ..hip import rng
from ..hip.conv import conv2d, conv_transpose2d
from ..hip.linear import linear
from ..hip.norm import bn_snake, snake, snake_skip
from ..hip.signal import istft_decode, stft_encode
from ..utils import SnakeActivation
from ..utils.train_utils import band_of


def _a(snake_mod):
    return snake_mod.a  # the (1,C,1,1) Parameter: kernels read it flat, grads land in .grad


class ResBlock(nn.Module):
    """vq_vae.py:13-62."""

    def __init__(self, in_channels, out_channels, frequency_indepence: bool, mid_channels=None,
                 dropout: float = 0.0):
        super().__init__()
        if frequency_indepence:
            raise NotImplementedError("frequency_indepence=True is not on the path (stage1.py:42)")
        if mid_channels is None:
            mid_channels = out_channels
        kernel_size, padding = (3, 3), (1, 1)
        layers = [
            SnakeActivation(in_channels, 2),
            nn.Conv2d(in_channels, mid_channels, kernel_size=kernel_size, stride=(1, 1),
                      padding=padding),
            nn.BatchNorm2d(out_channels),
            SnakeActivation(out_channels, 2),
            nn.Conv2d(mid_channels, out_channels, kernel_size=kernel_size, stride=(1, 1),
                      padding=padding),
            nn.Dropout(dropout),
        ]
        self.convs = nn.Sequential(*layers)
        self.proj = (nn.Identity() if in_channels == out_channels
                     else nn.Conv2d(in_channels, out_channels, kernel_size=1))
        self._site = rng.new_site()

    def forward(self, x):
        c = self.convs
        s, xs = snake_skip(x, _a(c[0]))  # xs: x, its skip-path gradient summed in Snake bwd
        h = conv2d(s, c[1].weight, c[1].bias)
        h = bn_snake(h, c[2], _a(c[3]))
        r = xs if isinstance(self.proj, nn.Identity) else conv2d(xs, self.proj.weight, self.proj.bias)
        p = c[5].p if self.training else 0.0
        return conv2d(h, c[4].weight, c[4].bias, residual=r, drop_p=p, site=self._site)


class VQVAEEncBlock(nn.Module):
    """vq_vae.py:65-92."""

    def __init__(self, in_channels, out_channels, frequency_indepence: bool, dropout: float = 0.0):
        super().__init__()
        if frequency_indepence:
            raise NotImplementedError("frequency_indepence=True is not on the path")
        self.block = nn.Sequential(
            nn.Conv2d(in_channels, out_channels, kernel_size=(3, 4), stride=(1, 2),
                      padding=(1, 1), padding_mode="replicate"),
            nn.BatchNorm2d(out_channels),
            SnakeActivation(out_channels, 2),
            nn.Dropout(dropout),
        )

    def forward(self, x):
        b = self.block
        if self.training and b[3].p > 0:
            raise NotImplementedError("EncBlock dropout>0 is not on the path (vq_vae.py:156)")
        h = conv2d(x, b[0].weight, b[0].bias, stride_w=2, replicate=True)
        return bn_snake(h, b[1], _a(b[2]))


class VQVAEDecBlock(nn.Module):
    """vq_vae.py:95-121."""

    def __init__(self, in_channels, out_channels, frequency_indepence: bool, dropout: float = 0.0):
        super().__init__()
        if frequency_indepence:
            raise NotImplementedError("frequency_indepence=True is not on the path")
        self.block = nn.Sequential(
            nn.ConvTranspose2d(in_channels, out_channels, kernel_size=(3, 4), stride=(1, 2),
                               padding=(1, 1)),
            nn.BatchNorm2d(out_channels),
            SnakeActivation(out_channels, 2),
            nn.Dropout(dropout),
        )

    def forward(self, x):
        b = self.block
        if self.training and b[3].p > 0:
            raise NotImplementedError("DecBlock dropout>0 is not on the path")
        h = conv_transpose2d(x, b[0].weight, b[0].bias, stride_w=2)
        return bn_snake(h, b[1], _a(b[2]))


class VQVAEEncoder(nn.Module):
    """vq_vae.py:124-188."""

    def __init__(self, init_dim: int, hid_dim: int, num_channels: int, downsample_rate: int,
                 n_resnet_blocks: int, pad_func, n_fft: int, frequency_indepence: bool,
                 dropout: float = 0.3, **kwargs):
        super().__init__()
        if n_fft != 4:
            raise NotImplementedError("n_fft=4 only (config.yaml VQ-VAE.n_fft)")
        self.pad_func = pad_func
        self.band = band_of(pad_func)
        self.n_fft = n_fft
        d = init_dim
        enc_layers = [VQVAEEncBlock(num_channels, d, frequency_indepence)]
        d *= 2
        for _ in range(int(round(np.log2(downsample_rate))) - 1):
            enc_layers.append(VQVAEEncBlock(d // 2, d, frequency_indepence))
            for _ in range(n_resnet_blocks):
                enc_layers.append(ResBlock(d, d, frequency_indepence, dropout=dropout))
            d *= 2
        enc_layers.append(ResBlock(d // 2, hid_dim, frequency_indepence, dropout=dropout))
        self.encoder = nn.Sequential(*enc_layers)
        self.is_num_tokens_updated = False
        self.register_buffer("num_tokens", torch.tensor(0))
        self.register_buffer("H_prime", torch.tensor(0))
        self.register_buffer("W_prime", torch.tensor(0))

    def encode_timefreq(self, u):
        """Run the conv stack on a band-copied STFT image u (B, 2C, 3, T+1)."""
        out = u
        for layer in self.encoder:
            out = layer(out)
        if not self.is_num_tokens_updated:
            self.H_prime = torch.tensor(out.shape[2])
            self.W_prime = torch.tensor(out.shape[3])
            self.num_tokens = self.H_prime * self.W_prime
            self.is_num_tokens_updated = True
        return out

    def forward(self, x):
        """x: (b c l) -> (b hid 3 W')."""
        key = "enc_l" if self.band == "lf" else "enc_h"
        u = stft_encode(x, **{key: True})[key]
        return self.encode_timefreq(u)


class VQVAEDecoder(nn.Module):
    """vq_vae.py:191-264."""

    def __init__(self, init_dim: int, hid_dim: int, num_channels: int, downsample_rate: int,
                 n_resnet_blocks: int, input_length: int, pad_func, n_fft: int, x_channels: int,
                 frequency_indepence: bool, dropout: float = 0.3, **kwargs):
        super().__init__()
        if n_fft != 4:
            raise NotImplementedError("n_fft=4 only")
        self.pad_func = pad_func
        self.band = band_of(pad_func)
        self.n_fft = n_fft
        self.x_channels = x_channels
        self.input_length = input_length
        kernel_size, padding = (3, 4), (1, 1)
        d = int(init_dim * 2 ** (int(round(np.log2(downsample_rate))) - 1))
        if round(np.log2(downsample_rate)) == 0:
            d = int(init_dim * 2 ** (int(round(np.log2(downsample_rate)))))
        dec_layers = [ResBlock(hid_dim, d, frequency_indepence, dropout=dropout)]
        for _ in range(int(round(np.log2(downsample_rate))) - 1):
            for _ in range(n_resnet_blocks):
                dec_layers.append(ResBlock(d, d, frequency_indepence, dropout=dropout))
            d //= 2
            dec_layers.append(VQVAEDecBlock(2 * d, d, frequency_indepence))
        dec_layers.append(nn.ConvTranspose2d(d, num_channels, kernel_size=kernel_size,
                                             stride=(1, 2), padding=padding))
        dec_layers.append(nn.ConvTranspose2d(num_channels, num_channels, kernel_size=kernel_size,
                                             stride=(1, 2), padding=padding))
        self.decoder = nn.Sequential(*dec_layers)
        self.interp = nn.Upsample(input_length, mode="linear")
        self.linear = nn.Linear(input_length, input_length)

    def forward(self, x):
        out = x
        for layer in self.decoder:
            if isinstance(layer, nn.ConvTranspose2d):
                out = conv_transpose2d(out, layer.weight, layer.bias, stride_w=2)
            else:
                out = layer(out)
        out = istft_decode(out, self.x_channels, self.band, self.input_length)  # (b c l)
        return linear(out, self.linear.weight, self.linear.bias, residual=out)
