"""FidelityEnhancer (reference models/fidelity_enhancer.py:458-498) and its 1-D U-Net
(:289-455), eval forward on the HIP path (csrc/tvq_fe.hip via hip/fe.py).

Only the parameter layout is taken from the reference: attribute names and container
indices reproduce its state_dict keys, so `stage3.ckpt`'s `fidelity_enhancer.*` entries
load unchanged (generation/sampler.py:94-106).  The modules here are thin parameter
holders; each forward is a handful of fused launches:

  ResNet unit  (:207-231)  ws-conv3 -> [GroupNorm+Snake] -> ws-conv3 -> [GroupNorm+Snake
                            + skip], the skip a 1x1 conv or the input itself
  linear attn  (:234-260)  [channel LN] -> [to_qkv + attention core, q/k/v in LDS]
                            -> 1x1 conv -> [channel LN + residual]
  full attn    (:263-283)  [channel LN] -> 1x1 conv -> [attention] -> [1x1 conv + residual]
  up-sampling  (:85-89)     nearest x2 read inside the following conv3
  skips        (:434-452)  [interpolate + concat] in one launch

No time embedding reaches the network (Unet1D.forward never passes one), and Dropout is
the identity in eval mode.

Training mode (Stage3, trainers/stage3.py:197-231) runs the same graph through
differentiable ops (hip/fe_train.py): the convolutions on the conv engine (H = 1, fused
bias / residual, deterministic weight gradients), the weight standardisation, GroupNorm +
Snake + the Block's Dropout (counter-hash mask, site per Block), channel LayerNorm, both
attention cores and the interpolate+concat skips, each with a HIP backward.
"""
import math

import torch
import torch.nn as nn

from ..hip import fe as ops
from ..hip import fe_train as tops
from ..hip import rng
from ..hip.conv import conv2d
from ..hip.xf import upsample_nearest
from ..utils import SnakeActivation

_EPS = 1e-5  # the reference's fp32 eps for weight standardisation, LN and GroupNorm


def _train(module):
    """Training graph: the module is in training mode and autograd is recording."""
    return module.training and torch.is_grad_enabled()


class _Conv(nn.Conv1d):
    """A Conv1d whose forward is tvq_fe_conv1d (any stride, zero or replicate padding,
    optional nearest-x2 input, optional fused residual)."""

    def __init__(self, cin, cout, k, stride=1, pad=0, replicate=False, upsample2=False,
                 bias=True):
        super().__init__(cin, cout, k, stride, pad, bias=bias,
                         padding_mode="replicate" if replicate else "zeros")
        self._up2 = upsample2

    def forward(self, x, residual=None):
        if _train(self):
            return self._train_forward(x, self.weight, residual)
        return ops.conv1d(x, self.weight, self.bias, stride=self.stride[0],
                          padding=self.padding[0], upsample2=self._up2,
                          replicate=self.padding_mode == "replicate", residual=residual)

    def _train_forward(self, x, w, residual=None):
        k = self.kernel_size[0]
        if self.padding[0] != (k - 1) // 2:
            raise NotImplementedError(f"conv1d k{k} pad {self.padding[0]} is not on the path")
        if self._up2:
            x = upsample_nearest(x, 2 * x.shape[-1])
        return conv2d(x, w, self.bias, stride_w=self.stride[0],
                      replicate=self.padding_mode == "replicate", residual=residual)


class _StandardizedConv(nn.Conv1d):
    """Weight-standardised conv3 (:96-116).  Eager: the standardised weight is recomputed
    only when the parameter changes (its version counter moves on every in-place update
    through the parameter; writes through `.data` do not move it, so call
    `invalidate()` after those).  Under hipGraph capture it is always recomputed inside
    the graph, so replays read the weight as it is at replay time."""

    def __init__(self, cin, cout):
        super().__init__(cin, cout, 3, padding=1)

    def invalidate(self):
        self._ws_key = None

    def forward(self, x):
        if _train(self):
            self._ws_key = None
            return conv2d(x, tops.standardize_weight(self.weight, _EPS), self.bias)
        key = (self.weight.data_ptr(), self.weight._version, self.weight.device)
        if torch.cuda.is_current_stream_capturing():
            self._ws_key = None
            return ops.conv1d(x, ops.standardize_weight(self.weight, _EPS), self.bias, padding=1)
        if getattr(self, "_ws_key", None) != key:
            self._ws = ops.standardize_weight(self.weight, _EPS)
            self._ws_key = key
        return ops.conv1d(x, self._ws, self.bias, padding=1)


class _Identity(nn.Module):
    """Parameter-free slot (nearest x2 folded into the next conv; the time embedding's
    sinusoid) that keeps the reference's container indices."""

    def forward(self, x, *args, **kwargs):
        return x


class _ChannelNorm(nn.Module):
    """Channel LayerNorm with gain `g` (1, C, 1) (:119-127)."""

    def __init__(self, channels):
        super().__init__()
        self.g = nn.Parameter(torch.ones(1, channels, 1))

    def forward(self, x, residual=None):
        if _train(self):
            return tops.channel_layernorm(x, self.g, _EPS, residual=residual)
        return ops.channel_layernorm(x, self.g, _EPS, residual=residual)


class _ConvNormAct(nn.Module):
    """conv -> GroupNorm -> Snake (-> Dropout, identity in eval) (:182-204); the unit's
    skip add rides in the GroupNorm+Snake kernel."""

    def __init__(self, cin, cout, groups, dropout):
        super().__init__()
        self.proj = _StandardizedConv(cin, cout)
        self.norm = nn.GroupNorm(groups, cout)
        self.act = SnakeActivation(cout, dim=1)
        self.dropout = nn.Dropout(dropout)
        self._site = rng.new_site()

    def forward(self, x, residual=None):
        if _train(self):
            return tops.group_norm_snake(self.proj(x), self.norm.num_groups, self.norm.weight,
                                         self.norm.bias, self.act.a, self.norm.eps,
                                         residual=residual, drop_p=self.dropout.p,
                                         site=self._site)
        return ops.group_norm_snake(self.proj(x), self.norm.num_groups, self.norm.weight,
                                    self.norm.bias, self.act.a, self.norm.eps,
                                    residual=residual)


class _ResUnit(nn.Module):
    """ResnetBlock (:207-231).  `mlp` holds the time-conditioning weights (never used by
    the forward the reference runs; kept for the state_dict)."""

    def __init__(self, cin, cout, time_dim, groups, dropout):
        super().__init__()
        self.mlp = nn.Sequential(nn.SiLU(), nn.Linear(time_dim, 2 * cout))
        self.block1 = _ConvNormAct(cin, cout, groups, dropout)
        self.block2 = _ConvNormAct(cout, cout, groups, dropout)
        self.res_conv = _Conv(cin, cout, 1) if cin != cout else _Identity()

    def forward(self, x):
        return self.block2(self.block1(x), residual=self.res_conv(x))


class _LinearAttnCore(nn.Module):
    """to_qkv / to_out of LinearAttention (:234-260): 4 heads of 32."""

    def __init__(self, channels, heads=4, dim_head=32):
        super().__init__()
        self.heads, self.dim_head = heads, dim_head
        self.to_qkv = nn.Conv1d(channels, 3 * heads * dim_head, 1, bias=False)
        self.to_out = nn.Sequential(nn.Conv1d(heads * dim_head, channels, 1),
                                    _ChannelNorm(channels))

    def forward(self, xn, residual):
        proj, norm = self.to_out
        if _train(self):
            att = tops.linear_attention(conv2d(xn, self.to_qkv.weight), self.heads, self.dim_head)
            return norm(conv2d(att, proj.weight, proj.bias), residual=residual)
        att = ops.linear_attention_fused(xn, self.to_qkv.weight, self.heads, self.dim_head)
        return norm(ops.conv1d(att, proj.weight, proj.bias), residual=residual)


class _FullAttnCore(nn.Module):
    """to_qkv / to_out of Attention (:263-283): 4 heads of 32, exact softmax."""

    def __init__(self, channels, heads=4, dim_head=32):
        super().__init__()
        self.heads, self.dim_head = heads, dim_head
        self.to_qkv = nn.Conv1d(channels, 3 * heads * dim_head, 1, bias=False)
        self.to_out = nn.Conv1d(heads * dim_head, channels, 1)

    def forward(self, xn, residual):
        if _train(self):
            att = tops.attention(conv2d(xn, self.to_qkv.weight), self.heads, self.dim_head)
            return conv2d(att, self.to_out.weight, self.to_out.bias, residual=residual)
        att = ops.attention(ops.conv1d(xn, self.to_qkv.weight), self.heads, self.dim_head)
        return ops.conv1d(att, self.to_out.weight, self.to_out.bias, residual=residual)


class _NormedResidual(nn.Module):
    """Residual(PreNorm(core)) (:75-82, :130-137) as one module: `fn.norm`, `fn.fn`."""

    class _Pre(nn.Module):
        def __init__(self, channels, core):
            super().__init__()
            self.fn = core
            self.norm = _ChannelNorm(channels)

    def __init__(self, channels, core):
        super().__init__()
        self.fn = self._Pre(channels, core)

    def forward(self, x):
        return self.fn.fn(self.fn.norm(x), residual=x)


class _TimeFourier(nn.Module):
    """Learned / random Fourier features of the time embedding (:158-176); present only
    for configs with learned_sinusoidal_cond, for their `weights` key."""

    def __init__(self, dim, frozen):
        super().__init__()
        self.weights = nn.Parameter(torch.randn(dim // 2), requires_grad=not frozen)

    def forward(self, t):
        f = t[:, None] * self.weights[None, :] * (2 * math.pi)
        return torch.cat((t[:, None], f.sin(), f.cos()), dim=-1)


def _upsampler(cin, cout):
    """Upsample (:85-89): [nearest x2 (folded), conv3 reading the upsampled input]."""
    return nn.Sequential(_Identity(), _Conv(cin, cout, 3, pad=1, upsample2=True))


class Unet1D(nn.Module):
    """Reference constructor signature (:289-304); the layer plan is derived from `dims`
    level by level (encoder: two ResNet units, linear attention, stride-2 conv4 or a conv3 at
    the last level; decoder mirrored with concatenated skips and x2 up-sampling)."""

    def __init__(self, dim, init_dim=None, out_dim=None, dim_mults=(1, 2, 4, 8), channels=1,
                 self_condition=False, resnet_block_groups=8, learned_variance=False,
                 learned_sinusoidal_cond=False, random_fourier_features=False,
                 learned_sinusoidal_dim=16, dropout: float = 0.0, **kwargs):
        super().__init__()
        self.channels, self.self_condition = channels, self_condition
        init_dim = dim if init_dim is None else init_dim
        widths = [init_dim] + [dim * m for m in dim_mults]
        pairs = list(zip(widths[:-1], widths[1:]))
        tdim = 4 * dim
        unit = lambda cin, cout: _ResUnit(cin, cout, tdim, resnet_block_groups, dropout)  # noqa: E731

        self.init_conv = _Conv(channels * (2 if self_condition else 1), init_dim, 7, pad=3)
        fourier = learned_sinusoidal_cond or random_fourier_features
        self.random_or_learned_sinusoidal_cond = fourier
        emb, emb_dim = ((_TimeFourier(learned_sinusoidal_dim, random_fourier_features),
                         learned_sinusoidal_dim + 1) if fourier else (_Identity(), dim))
        self.time_mlp = nn.Sequential(emb, nn.Linear(emb_dim, tdim), nn.GELU(),
                                      nn.Linear(tdim, tdim))

        last = len(pairs) - 1
        self.downs = nn.ModuleList(
            nn.ModuleList([unit(a, a), unit(a, a), _NormedResidual(a, _LinearAttnCore(a)),
                           _Conv(a, b, 4, 2, 1) if lvl < last else _Conv(a, b, 3, pad=1)])
            for lvl, (a, b) in enumerate(pairs))
        mid = widths[-1]
        self.mid_block1 = unit(mid, mid)
        self.mid_attn = _NormedResidual(mid, _FullAttnCore(mid))
        self.mid_block2 = unit(mid, mid)
        self.ups = nn.ModuleList(
            nn.ModuleList([unit(b + a, b), unit(b + a, b), _NormedResidual(b, _LinearAttnCore(b)),
                           _upsampler(b, a) if lvl < last else _Conv(b, a, 3, pad=1)])
            for lvl, (a, b) in enumerate(reversed(pairs)))
        self.last_up = _upsampler(pairs[0][0], pairs[0][0])
        self.out_dim = out_dim if out_dim is not None else channels * (2 if learned_variance else 1)
        self.final_res_block = unit(2 * dim, dim)
        self.final_conv = nn.Sequential(
            _Conv(dim, self.out_dim, 1),
            _Conv(self.out_dim, self.out_dim, 3, pad=1, replicate=True),
            _Conv(self.out_dim, self.out_dim, 3, pad=1, replicate=True))

    def forward(self, x):
        cat = tops.cat_interp if _train(self) else ops.cat_interp
        x = self.init_conv(x)
        stem, skips = x, []
        for res1, res2, attn, down in self.downs:
            x = res1(x)
            skips.append(x)
            x = attn(res2(x))
            skips.append(x)
            x = down(x)
        x = self.mid_block2(self.mid_attn(self.mid_block1(x)))
        for res1, res2, attn, up in self.ups:
            x = res1(cat(x, skips.pop(), x.shape[-1]))
            x = res2(cat(x, skips.pop(), x.shape[-1]))
            x = up(attn(x))
        x = self.final_res_block(cat(self.last_up(x), stem, stem.shape[-1]))
        return self.final_conv(x)


class FidelityEnhancer(nn.Module):
    """x_a (b, c, l) -> refined (b, c, input_length) (:458-498)."""

    def __init__(self, input_length, in_channels, config):
        super().__init__()
        self.input_length = input_length
        self.unet = Unet1D(channels=in_channels, **config["fidelity_enhancer"])
        self.register_buffer("tau", torch.tensor(0.0).float())

    def forward(self, x_a):
        """Eval: no autograd (the sampler's use).  Training: differentiable in the FE's
        parameters (Stage3)."""
        x_a = x_a.float()
        if _train(self):
            if x_a.shape[-1] != self.input_length:
                x_a = tops.cat_interp(x_a, None, self.input_length)
            return self.unet(x_a)
        with torch.no_grad():
            if x_a.shape[-1] != self.input_length:
                x_a = ops.cat_interp(x_a, None, self.input_length)
            return self.unet(x_a)
