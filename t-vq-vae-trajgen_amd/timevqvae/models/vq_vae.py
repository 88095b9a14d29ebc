"""Stage1 encoder/decoder — same API and module tree as the reference
timevqvae/models/vq_vae.py (state_dict keys `encoder.{i}.block.0.weight`,
`convs.{0..5}`, `proj`, `decoder.{i}`, `linear` ... are identical), executed by
the HIP kernels:

  VQVAEEncBlock  replicate-pad Conv2d(3x4, s(1,2)) with the BN statistics in its epilogue
                 -> [BN finish + apply + Snake in one launch]
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

from ..hip import resblock, rng
from ..hip.conv import (bn_eval_fusable, bnstats_blocks, conv2d, conv2d_bn_eval,
                        conv2d_bnstats, conv_transpose2d, conv_transpose2d_bn_eval,
                        conv_transpose2d_bnstats)
from ..hip.linear import linear
from ..hip.norm import bn_snake, bn_snake_part, snake, snake_skip
from ..hip.signal import istft_decode, stft_encode
from ..utils import SnakeActivation
from ..utils.train_utils import band_of


# training Enc/DecBlocks: the BatchNorm statistics in the stride-2 conv's epilogue
# (tvq_conv2d_fwd_bnstats + tvq_bn_train_apply_part); False (tests): conv, then the BN's
# own passes
BN_STATS_IN_CONV = True


def _a(snake_mod):
    return snake_mod.a  # the (1,C,1,1) Parameter: kernels read it flat, grads land in .grad


def _no_freq_indep(flag):
    if flag:
        raise NotImplementedError("frequency_indepence=True is not on the path (stage1.py:42)")


def _conv3x3(cin, cout):
    return nn.Conv2d(cin, cout, kernel_size=(3, 3), stride=(1, 1), padding=(1, 1))


def _strided_block(conv, cout, dropout):
    """[conv (3x4, stride (1,2)), BN, Snake, Dropout] as EncBlock / DecBlock hold it."""
    return nn.Sequential(conv, nn.BatchNorm2d(cout), SnakeActivation(cout, 2), nn.Dropout(dropout))


def _n_levels(downsample_rate):
    return int(round(np.log2(downsample_rate)))


def _encoder_plan(init_dim, hid_dim, num_channels, downsample_rate, n_res):
    """(kind, cin, cout) per layer of VQVAEEncoder.encoder (vq_vae.py:143-170): a strided
    block per octave of the rate, n_res ResBlocks after every one but the first, then the
    ResBlock into hid_dim."""
    plan, width = [("down", num_channels, init_dim)], init_dim
    for _ in range(_n_levels(downsample_rate) - 1):
        plan.append(("down", width, 2 * width))
        width *= 2
        plan += [("res", width, width)] * n_res
    return plan + [("res", width, hid_dim)]


def _decoder_plan(init_dim, hid_dim, num_channels, downsample_rate, n_res):
    """(kind, cin, cout) per layer of VQVAEDecoder.decoder (vq_vae.py:211-251): ResBlock out
    of hid_dim, then per octave n_res ResBlocks and a transposed strided block halving the
    width, then two transposed convs to num_channels."""
    lv = _n_levels(downsample_rate)
    width = int(init_dim * 2 ** (lv - 1)) if lv != 0 else int(init_dim)
    plan = [("res", hid_dim, width)]
    for _ in range(lv - 1):
        plan += [("res", width, width)] * n_res
        plan.append(("up", width, width // 2))
        width //= 2
    return plan + [("convT", width, num_channels), ("convT", num_channels, num_channels)]


class ResBlock(nn.Module):
    """vq_vae.py:13-62."""

    def __init__(self, in_channels, out_channels, frequency_indepence: bool, mid_channels=None,
                 dropout: float = 0.0):
        super().__init__()
        _no_freq_indep(frequency_indepence)
        mid = out_channels if mid_channels is None else mid_channels
        # convs: [Snake(in), conv3x3 in->mid, BN(out), Snake(out), conv3x3 mid->out, Dropout]
        self.convs = nn.Sequential(
            SnakeActivation(in_channels, 2), _conv3x3(in_channels, mid), nn.BatchNorm2d(out_channels),
            SnakeActivation(out_channels, 2), _conv3x3(mid, out_channels), nn.Dropout(dropout))
        self.proj = (nn.Conv2d(in_channels, out_channels, kernel_size=1)
                     if in_channels != out_channels else nn.Identity())
        self._site = rng.new_site()

    def fused_train_p(self, x):
        """The dropout p of the fused identity training path when it applies to x, else None."""
        c = self.convs
        if (isinstance(self.proj, nn.Identity) and c[2].training
                and resblock.supported(x, c[1].in_channels, c[4].out_channels)):
            return c[5].p if self.training else 0.0
        return None

    def forward(self, x):
        c = self.convs
        if isinstance(self.proj, nn.Identity) and resblock.supported(x, c[1].in_channels,
                                                                     c[4].out_channels):
            # the whole block as 2 (eval: 1) fused launches, csrc/tvq_resblock.hip
            if c[2].training:
                p = c[5].p if self.training else 0.0
                return resblock.resblock_train(x, _a(c[0]), c[1], c[2], _a(c[3]), c[4], p,
                                               self._site)
            # the fused eval launch builds no graph: only when nothing here needs a gradient
            # (an eval-mode block whose conv / BN / Snake parameters train takes the
            # autograd path below)
            needs_grad = torch.is_grad_enabled() and (
                x.requires_grad or any(p.requires_grad for p in self.parameters()))
            if not needs_grad and not (self.training and c[5].p > 0):
                return resblock.resblock_eval(x, _a(c[0]), c[1], c[2], _a(c[3]), c[4])
        if (not isinstance(self.proj, nn.Identity) and self.proj.bias is not None
                and resblock.proj_supported(x, c[1].in_channels, c[4].out_channels)):
            # the projection block as 2 (eval: 1) fused launches, csrc/tvq_resblock_w8p.hip
            if c[2].training:
                p = c[5].p if self.training else 0.0
                return resblock.resblock_proj_train(x, _a(c[0]), c[1], c[2], _a(c[3]), c[4],
                                                    self.proj, p, self._site)
            needs_grad = torch.is_grad_enabled() and (
                x.requires_grad or any(p.requires_grad for p in self.parameters()))
            if not needs_grad and not (self.training and c[5].p > 0):
                return resblock.resblock_proj_eval(x, _a(c[0]), c[1], c[2], _a(c[3]), c[4],
                                                   self.proj)
        s, xs = snake_skip(x, _a(c[0]))  # xs: x, its skip-path gradient summed in Snake bwd
        if bn_eval_fusable(s, c[2], c[1].weight, c[1].bias, c[3].a):
            h = conv2d_bn_eval(s, c[1].weight, c[1].bias, c[2], _a(c[3]))  # one launch
        else:
            h = conv2d(s, c[1].weight, c[1].bias)
            h = bn_snake(h, c[2], _a(c[3]))
        r = xs if isinstance(self.proj, nn.Identity) else conv2d(xs, self.proj.weight, self.proj.bias)
        p = c[5].p if self.training else 0.0
        return conv2d(h, c[4].weight, c[4].bias, residual=r, drop_p=p, site=self._site)


def _pairable(l1, l2, x):
    """Two consecutive identity ResBlocks that take the fused training path with equal
    dropout and BN hyper-parameters (run as one resblock.resblock_pair_train chain)."""
    if not (isinstance(l1, ResBlock) and isinstance(l2, ResBlock)):
        return None
    p1 = l1.fused_train_p(x)
    if p1 is None or p1 != l2.fused_train_p(x) or not resblock.pair_supported(x):
        return None
    b1, b2 = l1.convs[2], l2.convs[2]
    if b1.momentum != b2.momentum or b1.eps != b2.eps or b1.momentum is None:
        return None
    return p1


def run_layers(layers, x, layer_fn):
    """layer_fn over layers in order, consecutive pairable ResBlocks as one fused pair."""
    i, n = 0, len(layers)
    while i < n:
        p = _pairable(layers[i], layers[i + 1], x) if i + 1 < n else None
        if p is not None:
            x = resblock.resblock_pair_train(x, layers[i], layers[i + 1], p)
            i += 2
        else:
            x = layer_fn(layers[i], x)
            i += 1
    return x


def _call(layer, x):
    return layer(x)


class VQVAEEncBlock(nn.Module):
    """vq_vae.py:65-92."""

    def __init__(self, in_channels, out_channels, frequency_indepence: bool, dropout: float = 0.0):
        super().__init__()
        _no_freq_indep(frequency_indepence)
        self.block = _strided_block(
            nn.Conv2d(in_channels, out_channels, (3, 4), (1, 2), (1, 1), padding_mode="replicate"),
            out_channels, dropout)

    def forward(self, x):
        b = self.block
        if self.training and b[3].p > 0:
            raise NotImplementedError("EncBlock dropout>0 is not on the path (vq_vae.py:156)")
        if bn_eval_fusable(x, b[1], b[0].weight, b[0].bias, b[2].a):
            return conv2d_bn_eval(x, b[0].weight, b[0].bias, b[1], _a(b[2]), stride_w=2,
                                  replicate=True)
        if self.training and BN_STATS_IN_CONV and bnstats_blocks(x, b[0].weight, 2, False):
            # the BN statistics in the conv's epilogue, finished by the apply launch
            h, part = conv2d_bnstats(x, b[0].weight, b[0].bias, stride_w=2, replicate=True)
            return bn_snake_part(h, part, b[1], _a(b[2]))
        h = conv2d(x, b[0].weight, b[0].bias, stride_w=2, replicate=True)
        return bn_snake(h, b[1], _a(b[2]))


class VQVAEDecBlock(nn.Module):
    """vq_vae.py:95-121."""

    def __init__(self, in_channels, out_channels, frequency_indepence: bool, dropout: float = 0.0):
        super().__init__()
        _no_freq_indep(frequency_indepence)
        self.block = _strided_block(nn.ConvTranspose2d(in_channels, out_channels, (3, 4), (1, 2), (1, 1)),
                                    out_channels, dropout)

    def forward(self, x):
        b = self.block
        if self.training and b[3].p > 0:
            raise NotImplementedError("DecBlock dropout>0 is not on the path")
        if bn_eval_fusable(x, b[1], b[0].weight, b[0].bias, b[2].a):
            return conv_transpose2d_bn_eval(x, b[0].weight, b[0].bias, b[1], _a(b[2]))
        if self.training and BN_STATS_IN_CONV and bnstats_blocks(x, b[0].weight, 2, True):
            h, part = conv_transpose2d_bnstats(x, b[0].weight, b[0].bias, stride_w=2)
            return bn_snake_part(h, part, b[1], _a(b[2]))
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
        self.encoder = nn.Sequential(*(
            VQVAEEncBlock(cin, cout, frequency_indepence) if kind == "down"
            else ResBlock(cin, cout, frequency_indepence, dropout=dropout)
            for kind, cin, cout in _encoder_plan(init_dim, hid_dim, num_channels,
                                                 downsample_rate, n_resnet_blocks)))
        self.is_num_tokens_updated = False
        self.register_buffer("num_tokens", torch.tensor(0))
        self.register_buffer("H_prime", torch.tensor(0))
        self.register_buffer("W_prime", torch.tensor(0))

    def encode_timefreq(self, u):
        """Run the conv stack on a band-copied STFT image u (B, 2C, 3, T+1)."""
        out = run_layers(self.encoder, u, _call)
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
        make = {"res": lambda a, b: ResBlock(a, b, frequency_indepence, dropout=dropout),
                "up": lambda a, b: VQVAEDecBlock(a, b, frequency_indepence),
                "convT": lambda a, b: nn.ConvTranspose2d(a, b, (3, 4), (1, 2), (1, 1))}
        self.decoder = nn.Sequential(*(
            make[kind](cin, cout) for kind, cin, cout in _decoder_plan(
                init_dim, hid_dim, num_channels, downsample_rate, n_resnet_blocks)))
        self.interp = nn.Upsample(input_length, mode="linear")
        self.linear = nn.Linear(input_length, input_length)

    @staticmethod
    def _layer(layer, x):
        if isinstance(layer, nn.ConvTranspose2d):
            return conv_transpose2d(x, layer.weight, layer.bias, stride_w=2)
        return layer(x)

    def forward(self, x):
        out = run_layers(self.decoder, x, self._layer)
        out = istft_decode(out, self.x_channels, self.band, self.input_length)  # (b c l)
        return linear(out, self.linear.weight, self.linear.bias, residual=out)
