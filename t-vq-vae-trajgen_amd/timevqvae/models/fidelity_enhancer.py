"""FidelityEnhancer and its Unet1D (reference models/fidelity_enhancer.py) on the HIP path.

The module tree, constructor arguments and state_dict keys are the reference's, so a
reference `stage3.ckpt`'s `fidelity_enhancer.*` entries load unchanged
(generation/sampler.py:94-106).  The forward is the eval-mode forward (Dropout is the
identity, no time embedding: Unet1D.forward never passes one, :395-455) and runs on
csrc/tvq_fe.hip through hip/fe.py: weight-standardised convs, GroupNorm+Snake with the
ResnetBlock skip fused, channel LayerNorm with the Residual add fused, linear / full
attention, nearest-x2 upsampling read inside the conv, and interpolate+concat skips.
Training the FidelityEnhancer (Stage3) is not on the HIP path: forward raises in
training mode rather than silently differing from the reference's dropout."""
import math
from functools import partial

import torch
import torch.nn as nn

from ..hip import fe as ops
from ..utils import SnakeActivation


def exists(x):
    return x is not None


def default(val, d):
    if exists(val):
        return val
    return d() if callable(d) else d


class Residual(nn.Module):
    """fidelity_enhancer.py:75-82; the add is fused into the wrapped op's last kernel."""

    def __init__(self, fn):
        super().__init__()
        self.fn = fn

    def forward(self, x, *args, **kwargs):
        return self.fn(x, *args, residual=x, **kwargs)


class _UpsampleConv(nn.Conv1d):
    """Conv1d that reads its input nearest-upsampled by 2 (Upsample's two ops, :85-89)."""

    def forward(self, x):
        return ops.conv1d(x, self.weight, self.bias, padding=1, upsample2=True)


class _Nearest2(nn.Module):
    """nn.Upsample(scale_factor=2, mode="nearest") placeholder: parameter-free and folded
    into the following _UpsampleConv (keeps the Sequential's key indices)."""

    def forward(self, x):
        return x


def Upsample(dim, dim_out=None):
    return nn.Sequential(_Nearest2(), _UpsampleConv(dim, default(dim_out, dim), 3, padding=1))


class _Conv1d(nn.Conv1d):
    """nn.Conv1d on the HIP path (zero or replicate padding, any stride)."""

    def forward(self, x, residual=None):
        return ops.conv1d(x, self.weight, self.bias, stride=self.stride[0],
                          padding=self.padding[0], replicate=self.padding_mode == "replicate",
                          residual=residual)


def Downsample(dim, dim_out=None):
    return _Conv1d(dim, default(dim_out, dim), 4, 2, 1)


class WeightStandardizedConv2d(nn.Conv1d):
    """fidelity_enhancer.py:96-116 (the name is the reference's; it is a Conv1d)."""

    def forward(self, x):
        # the standardised weight is kept until the parameter changes (its version counter
        # moves on every in-place update: optimizer steps, load_state_dict, .to())
        key = (self.weight.data_ptr(), self.weight._version, self.weight.device)
        if getattr(self, "_ws_key", None) != key:
            self._ws = ops.standardize_weight(self.weight, 1e-5)
            self._ws_key = key
        return ops.conv1d(x, self._ws, self.bias, stride=self.stride[0], padding=self.padding[0])


class LayerNorm(nn.Module):
    """Channel LayerNorm, gamma only (:119-127)."""

    def __init__(self, dim):
        super().__init__()
        self.g = nn.Parameter(torch.ones(1, dim, 1))

    def forward(self, x, residual=None):
        return ops.channel_layernorm(x, self.g, 1e-5, residual=residual)


class PreNorm(nn.Module):
    """:130-137"""

    def __init__(self, dim, fn):
        super().__init__()
        self.fn = fn
        self.norm = LayerNorm(dim)

    def forward(self, x, residual=None):
        return self.fn(self.norm(x), residual=residual)


class SinusoidalPosEmb(nn.Module):
    """:143-155 (time embedding; parameter-free, unused by Unet1D.forward)."""

    def __init__(self, dim):
        super().__init__()
        self.dim = dim

    def forward(self, x):
        half_dim = self.dim // 2
        emb = math.log(10000) / (half_dim - 1)
        emb = torch.exp(torch.arange(half_dim, device=x.device) * -emb)
        emb = x[:, None] * emb[None, :]
        return torch.cat((emb.sin(), emb.cos()), dim=-1)


class RandomOrLearnedSinusoidalPosEmb(nn.Module):
    """:158-176 (kept for the state_dict layout of learned_sinusoidal_cond configs)."""

    def __init__(self, dim, is_random=False):
        super().__init__()
        assert (dim % 2) == 0
        self.weights = nn.Parameter(torch.randn(dim // 2), requires_grad=not is_random)

    def forward(self, x):
        x = x[:, None]
        freqs = x * self.weights[None, :] * 2 * math.pi
        return torch.cat((x, freqs.sin(), freqs.cos()), dim=-1)


class Block(nn.Module):
    """WS conv3 -> GroupNorm -> Snake -> Dropout (:182-204); the ResnetBlock's skip add
    rides in the GroupNorm+Snake kernel."""

    def __init__(self, dim, dim_out, groups=8, dropout=0.0):
        super().__init__()
        self.proj = WeightStandardizedConv2d(dim, dim_out, 3, padding=1)
        self.norm = nn.GroupNorm(groups, dim_out)
        self.act = SnakeActivation(dim_out, dim=1)
        self.dropout = nn.Dropout(dropout)

    def forward(self, x, scale_shift=None, residual=None):
        if scale_shift is not None:
            raise NotImplementedError("Block: scale_shift (time conditioning) is not on the HIP "
                                      "path; Unet1D.forward never passes it")
        x = self.proj(x)
        return ops.group_norm_snake(x, self.norm.num_groups, self.norm.weight, self.norm.bias,
                                    self.act.a, self.norm.eps, residual=residual)


class ResnetBlock(nn.Module):
    """:207-231 (time_emb never passed by Unet1D.forward; the mlp exists for the keys)."""

    def __init__(self, dim, dim_out, *, time_emb_dim=None, groups=8, dropout=0.0):
        super().__init__()
        self.mlp = (nn.Sequential(nn.SiLU(), nn.Linear(time_emb_dim, dim_out * 2))
                    if exists(time_emb_dim) else None)
        self.block1 = Block(dim, dim_out, groups=groups, dropout=dropout)
        self.block2 = Block(dim_out, dim_out, groups=groups, dropout=dropout)
        self.res_conv = _Conv1d(dim, dim_out, 1) if dim != dim_out else nn.Identity()

    def forward(self, x, time_emb=None):
        if time_emb is not None:
            raise NotImplementedError("ResnetBlock: time_emb is not on the HIP path")
        h = self.block1(x)
        return self.block2(h, residual=self.res_conv(x))


class LinearAttention(nn.Module):
    """:234-260"""

    def __init__(self, dim, heads=4, dim_head=32):
        super().__init__()
        self.scale = dim_head ** -0.5
        self.heads = heads
        self.dim_head = dim_head
        hidden_dim = dim_head * heads
        self.to_qkv = nn.Conv1d(dim, hidden_dim * 3, 1, bias=False)
        self.to_out = nn.Sequential(nn.Conv1d(hidden_dim, dim, 1), LayerNorm(dim))

    def forward(self, x, residual=None):
        out = ops.linear_attention_fused(x, self.to_qkv.weight, self.heads, self.dim_head)
        conv, norm = self.to_out
        return norm(ops.conv1d(out, conv.weight, conv.bias), residual=residual)


class Attention(nn.Module):
    """:263-283"""

    def __init__(self, dim, heads=4, dim_head=32):
        super().__init__()
        self.scale = dim_head ** -0.5
        self.heads = heads
        self.dim_head = dim_head
        hidden_dim = dim_head * heads
        self.to_qkv = nn.Conv1d(dim, hidden_dim * 3, 1, bias=False)
        self.to_out = nn.Conv1d(hidden_dim, dim, 1)

    def forward(self, x, residual=None):
        qkv = ops.conv1d(x, self.to_qkv.weight)
        out = ops.attention(qkv, self.heads, self.dim_head)
        return ops.conv1d(out, self.to_out.weight, self.to_out.bias, residual=residual)


class Unet1D(nn.Module):
    """:289-455, same constructor and module tree."""

    def __init__(self, dim, init_dim=None, out_dim=None, dim_mults=(1, 2, 4, 8), channels=1,
                 self_condition=False, resnet_block_groups=8, learned_variance=False,
                 learned_sinusoidal_cond=False, random_fourier_features=False,
                 learned_sinusoidal_dim=16, dropout: float = 0.0, **kwargs):
        super().__init__()
        self.channels = channels
        self.self_condition = self_condition
        input_channels = channels * (2 if self_condition else 1)
        init_dim = default(init_dim, dim)
        self.init_conv = _Conv1d(input_channels, init_dim, 7, padding=3)
        dims = [init_dim, *map(lambda m: dim * m, dim_mults)]
        in_out = list(zip(dims[:-1], dims[1:]))
        block_klass = partial(ResnetBlock, groups=resnet_block_groups, dropout=dropout)
        time_dim = dim * 4
        self.random_or_learned_sinusoidal_cond = learned_sinusoidal_cond or random_fourier_features
        if self.random_or_learned_sinusoidal_cond:
            sinu_pos_emb = RandomOrLearnedSinusoidalPosEmb(learned_sinusoidal_dim,
                                                           random_fourier_features)
            fourier_dim = learned_sinusoidal_dim + 1
        else:
            sinu_pos_emb = SinusoidalPosEmb(dim)
            fourier_dim = dim
        self.time_mlp = nn.Sequential(sinu_pos_emb, nn.Linear(fourier_dim, time_dim), nn.GELU(),
                                      nn.Linear(time_dim, time_dim))
        self.downs = nn.ModuleList([])
        self.ups = nn.ModuleList([])
        num_resolutions = len(in_out)
        for ind, (dim_in, dim_out) in enumerate(in_out):
            is_last = ind >= (num_resolutions - 1)
            self.downs.append(nn.ModuleList([
                block_klass(dim_in, dim_in, time_emb_dim=time_dim),
                block_klass(dim_in, dim_in, time_emb_dim=time_dim),
                Residual(PreNorm(dim_in, LinearAttention(dim_in))),
                Downsample(dim_in, dim_out) if not is_last else _Conv1d(dim_in, dim_out, 3, padding=1),
            ]))
        mid_dim = dims[-1]
        self.mid_block1 = block_klass(mid_dim, mid_dim, time_emb_dim=time_dim)
        self.mid_attn = Residual(PreNorm(mid_dim, Attention(mid_dim)))
        self.mid_block2 = block_klass(mid_dim, mid_dim, time_emb_dim=time_dim)
        for ind, (dim_in, dim_out) in enumerate(reversed(in_out)):
            is_last = ind == (len(in_out) - 1)
            self.ups.append(nn.ModuleList([
                block_klass(dim_out + dim_in, dim_out, time_emb_dim=time_dim),
                block_klass(dim_out + dim_in, dim_out, time_emb_dim=time_dim),
                Residual(PreNorm(dim_out, LinearAttention(dim_out))),
                Upsample(dim_out, dim_in) if not is_last else _Conv1d(dim_out, dim_in, 3, padding=1),
            ]))
        self.last_up = Upsample(dim_in, dim_in)
        default_out_dim = channels * (1 if not learned_variance else 2)
        self.out_dim = default(out_dim, default_out_dim)
        self.final_res_block = block_klass(dim * 2, dim, time_emb_dim=time_dim)
        self.final_conv = nn.Sequential(
            _Conv1d(dim, self.out_dim, kernel_size=1),
            _Conv1d(self.out_dim, self.out_dim, kernel_size=3, padding=1, padding_mode="replicate"),
            _Conv1d(self.out_dim, self.out_dim, kernel_size=3, padding=1, padding_mode="replicate"),
        )

    def forward(self, x):
        if self.training:
            raise NotImplementedError(
                "Unet1D: the HIP path implements the eval forward (the sampler's use); "
                "Stage3 training of the FidelityEnhancer is not on it (call .eval())")
        x = self.init_conv(x)
        r = x
        h = []
        for block1, block2, attn, downsample in self.downs:
            x = block1(x)
            h.append(x)
            x = block2(x)
            x = attn(x)
            h.append(x)
            x = downsample(x)
        x = self.mid_block1(x)
        x = self.mid_attn(x)
        x = self.mid_block2(x)
        for block1, block2, attn, upsample in self.ups:
            x = block1(ops.cat_interp(x, h.pop(), x.shape[-1]))
            x = block2(ops.cat_interp(x, h.pop(), x.shape[-1]))
            x = attn(x)
            x = upsample(x)
        x = self.last_up(x)
        x = self.final_res_block(ops.cat_interp(x, r, r.shape[-1]))
        return self.final_conv(x)


class FidelityEnhancer(nn.Module):
    """fidelity_enhancer.py:458-498: interpolate x_a to input_length, then the Unet1D."""

    def __init__(self, input_length, in_channels, config):
        super().__init__()
        self.input_length = input_length
        self.unet = Unet1D(channels=in_channels, **config["fidelity_enhancer"])
        self.register_buffer("tau", torch.tensor(0.0).float())

    @torch.no_grad()
    def forward(self, x_a):
        """x_a (b, c, l) -> (b, c, input_length)."""
        x_a = x_a.float()
        if x_a.shape[-1] != self.input_length:
            x_a = ops.cat_interp(x_a, None, self.input_length)
        return self.unet(x_a)
