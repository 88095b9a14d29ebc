"""Eval-mode conv -> BatchNorm -> Snake in one launch (tvq_conv2d_fwd_bn_eval /
tvq_convT2d_fwd_bn_eval; VQVAEDecBlock.block and ResBlock.convs[1:4] while sampling,
vq_vae.py:31-48,98-118) against the two-launch HIP path (conv, then tvq_bn_eval_fwd) and
against torch fp32 (F.conv2d / F.conv_transpose2d, F.batch_norm with the running
statistics, x + sin(a x)^2 / a).  The sampler's decoder shapes at B = 1024 must take a
fused epilogue (no "bn_eval separate" in the dispatch trace); other shapes may fall back to
the separate BN launch and must give the same numbers.  Tolerance: rel-L2 1e-6 against the
two-launch path (the fused Snake's sin^2 is a Cody-Waite / polynomial evaluation, ~1e-7
relative of sinf), 1e-5 against torch (conv summation order)."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).norm() / (b.norm() + 1e-30))


def _bn(C, cuda, seed):
    g = torch.Generator().manual_seed(seed)
    bn = nn.BatchNorm2d(C).to(cuda).eval()
    with torch.no_grad():
        bn.weight.copy_(torch.rand(C, generator=g) + 0.5)
        bn.bias.copy_(torch.randn(C, generator=g) * 0.3)
        bn.running_mean.copy_(torch.randn(C, generator=g) * 0.2)
        bn.running_var.copy_(torch.rand(C, generator=g) + 0.3)
    a = (torch.rand(1, C, 1, 1, generator=g) * 1.5 + 0.25).to(cuda)
    return bn, a


def _torch_ref(h, bn, a):
    y = F.batch_norm(h, bn.running_mean, bn.running_var, bn.weight, bn.bias, False, 0.0, bn.eps)
    return y + (1.0 / a) * torch.sin(a * y) ** 2 if a is not None else y


# (B, Ci, H, Wi, Co, transposed, must_fuse): the sampler's decoder convs feeding a BN at
# B = 1024 (LF ResBlock 128 -> 64 and 64 -> 64, HF ResBlock 128 -> 16, the DecBlocks),
# and small / odd shapes that take other conv paths
SHAPES = [
    (1024, 128, 3, 8, 64, False, True),
    (1024, 64, 3, 8, 64, False, True),
    (1024, 128, 3, 32, 16, False, True),
    (256, 16, 3, 32, 128, False, True),
    (1024, 64, 3, 8, 32, True, True),
    (1024, 32, 3, 16, 16, True, True),
    (1024, 16, 3, 32, 8, True, True),
    (1024, 8, 3, 64, 4, True, True),
    (256, 12, 3, 257, 4, "enc", True),
    (256, 4, 3, 129, 8, "enc", True),
    (256, 16, 3, 33, 32, "enc", True),
    (3, 8, 3, 17, 8, False, False),
    (5, 12, 3, 33, 12, True, False),
    (2, 64, 3, 8, 64, False, False),
]


@pytest.mark.parametrize("B,Ci,H,Wi,Co,tr,must_fuse", SHAPES)
@pytest.mark.parametrize("with_snake", [True, False])
def test_conv_bn_eval_matches_two_launches(B, Ci, H, Wi, Co, tr, must_fuse, with_snake, cuda):
    from timevqvae.hip._native import plan_trace
    from timevqvae.hip.conv import (conv2d, conv2d_bn_eval, conv_transpose2d,
                                    conv_transpose2d_bn_eval)
    from timevqvae.hip.norm import bn_snake
    torch.manual_seed(B + Ci + Co)
    x = torch.randn(B, Ci, H, Wi, device=cuda)
    enc = tr == "enc"  # EncBlock: replicate-padded 3x4 stride-2 conv
    tr = tr is True
    w = (torch.randn(Ci, Co, 3, 4) if tr else torch.randn(Co, Ci, 3, 4 if enc else 3)).to(cuda) * (Ci * 9) ** -0.5
    b = torch.randn(Co, device=cuda) * 0.1
    bn, a = _bn(Co, cuda, B + Co)
    a = a if with_snake else None
    with torch.no_grad():
        with plan_trace() as tr_:
            if enc:
                y = conv2d_bn_eval(x, w, b, bn, a, stride_w=2, replicate=True)
            else:
                y = conv_transpose2d_bn_eval(x, w, b, bn, a) if tr else conv2d_bn_eval(x, w, b, bn, a)
            torch.cuda.synchronize()
        if enc:
            h = conv2d(x, w, b, stride_w=2, replicate=True)
            hr = F.conv2d(F.pad(x, (1, 1, 1, 1), mode="replicate"), w, b, stride=(1, 2))
        else:
            h = conv_transpose2d(x, w, b) if tr else conv2d(x, w, b)
            hr = (F.conv_transpose2d(x, w, b, stride=(1, 2), padding=(1, 1)) if tr
                  else F.conv2d(x, w, b, padding=1))
        want = bn_snake(h, bn, a)
        ref = _torch_ref(hr, bn, a)
    sep = tr_.has("bn_eval separate")
    if must_fuse:
        assert not sep, tr_.lines
    assert y.shape == want.shape
    assert rel(y, want) < 1e-6, rel(y, want)
    assert rel(y, ref) < 1e-5, rel(y, ref)


@pytest.mark.parametrize("band", ["lf", "hf"])
def test_decoder_eval_uses_fused_blocks(band, cuda):
    """The config-B LF / HF decoders in eval mode at B = 64: the fused conv + BN launches give
    the same reconstruction as the per-op path (TVQ_FUSED_BN_EVAL off)."""
    from timevqvae.hip import conv as hconv
    from timevqvae.models.vq_vae import VQVAEDecoder
    from timevqvae.utils import zero_pad_high_freq, zero_pad_low_freq
    torch.manual_seed(0)
    rate, pad, W = (32, zero_pad_high_freq, 8) if band == "lf" else (8, zero_pad_low_freq, 32)
    dec = VQVAEDecoder(4, 128, 12, rate, 2, 256, pad, 4, 6, False).to(cuda).eval()
    with torch.no_grad():
        for m in dec.modules():
            if isinstance(m, nn.BatchNorm2d):
                m.running_mean.uniform_(-0.2, 0.2)
                m.running_var.uniform_(0.5, 1.5)
    z = torch.randn(64, 128, 3, W, device=cuda)
    with torch.no_grad():
        hconv.FUSED_BN_EVAL = True
        a = dec(z)
        hconv.FUSED_BN_EVAL = False
        try:
            b = dec(z)
        finally:
            hconv.FUSED_BN_EVAL = True
    assert rel(a, b) < 1e-5, rel(a, b)


@pytest.mark.parametrize("B,L", [(1024, 97), (7, 33)])
def test_conv1d_gelu_bn_eval(B, L, cuda):
    """Upscale's Conv1d(k3) -> GELU -> BatchNorm1d (bidirectional_transformer.py:37-52) as
    one launch (pre_gelu) against the three-launch HIP path and torch."""
    from timevqvae.hip._native import plan_trace
    from timevqvae.hip.conv import conv2d, conv2d_bn_eval
    from timevqvae.hip.norm import bn_snake
    from timevqvae.hip.xf import gelu
    torch.manual_seed(B)
    x = torch.randn(B, 128, L, device=cuda)
    w = torch.randn(128, 128, 3, device=cuda) * (128 * 3) ** -0.5
    b = torch.randn(128, device=cuda) * 0.1
    bn = nn.BatchNorm1d(128).to(cuda).eval()
    with torch.no_grad():
        bn.running_mean.uniform_(-0.2, 0.2)
        bn.running_var.uniform_(0.5, 1.5)
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.3, 0.3)
        with plan_trace() as tr_:
            y = conv2d_bn_eval(x, w, b, bn, None, pre_gelu=True)
            torch.cuda.synchronize()
        want = bn_snake(gelu(conv2d(x, w, b)), bn, None)
        ref = bn(F.gelu(F.conv1d(x, w, b, padding=1)))
    if B == 1024:
        assert not tr_.has("bn_eval separate"), tr_.lines
    assert rel(y, want) < 1e-6, rel(y, want)
    assert rel(y, ref) < 1e-5, rel(y, ref)
