"""Training Enc/DecBlocks with the BatchNorm statistics in the stride-2 conv's epilogue
(tvq_conv2d_fwd_bnstats + tvq_bn_train_apply_part; reference vq_vae.py:65-121: conv ->
BatchNorm2d -> Snake) at the step's B = 256 shapes, against (a) the separate conv + BN path of
this library and (b) torch CPU fp64 with train-mode BatchNorm.  The statistics are fp64 sums
in another order, so the bars are relative fp32 tolerances written per check."""
import copy

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

B = 256
# (kind, Ci, Co, input width): the EncBlocks 12 -> 4 -> 8 -> 16 and the DecBlocks 16 -> 8 -> 4
# of both bands at config B (BASELINE configs[1])
CASES = [("enc", 12, 4, 257), ("enc", 4, 8, 128), ("enc", 8, 16, 64), ("dec", 16, 8, 32),
         ("dec", 8, 4, 64), ("dec", 4, 4, 16)]


def _block(kind, Ci, Co, seed):
    from timevqvae.models.vq_vae import VQVAEDecBlock, VQVAEEncBlock
    torch.manual_seed(seed)
    m = (VQVAEEncBlock if kind == "enc" else VQVAEDecBlock)(Ci, Co, False)
    with torch.no_grad():
        m.block[1].weight.normal_(1.0, 0.3)
        m.block[1].bias.normal_(0.0, 0.3)
        m.block[1].running_mean.normal_()
        m.block[1].running_var.uniform_(0.5, 2.0)
        m.block[2].a.uniform_(0.3, 0.8)
    return m


def _ref(kind, m, x):
    """torch fp64: conv (replicate pad for the EncBlock) -> BatchNorm2d (train) -> Snake."""
    conv, bn, sn = m.block[0], m.block[1], m.block[2]
    w, b = conv.weight.double(), conv.bias.double()
    if kind == "enc":
        h = F.conv2d(F.pad(x, (1, 1, 1, 1), mode="replicate"), w, b, stride=(1, 2))
    else:
        h = F.conv_transpose2d(x, w, b, stride=(1, 2), padding=(1, 1))
    rm, rv = bn.running_mean.double().clone(), bn.running_var.double().clone()
    u = F.batch_norm(h, rm, rv, bn.weight.double(), bn.bias.double(), True, bn.momentum, bn.eps)
    a = sn.a.double()
    return u + (1.0 / a) * torch.sin(a * u) ** 2, rm, rv


@pytest.mark.parametrize("kind,Ci,Co,W", CASES)
def test_block_bn_stats_in_conv(kind, Ci, Co, W, cuda):
    from timevqvae.hip._native import plan_trace
    from timevqvae.hip.conv import bnstats_blocks
    from timevqvae.models import vq_vae
    m0 = _block(kind, Ci, Co, Ci * 100 + Co)
    gen = torch.Generator().manual_seed(W)
    x = torch.randn(B, Ci, 3, W, generator=gen) * 1.3
    runs = []
    for fused in (True, False):
        m = copy.deepcopy(m0).to(cuda).train()
        xd = x.to(cuda).requires_grad_(True)
        vq_vae.BN_STATS_IN_CONV = fused
        try:
            with plan_trace() as tr:
                y = m(xd)
                gy = torch.ones_like(y) + torch.linspace(-1, 1, y.numel(), device=cuda).view_as(y)
                y.backward(gy)
                torch.cuda.synchronize()
        finally:
            vq_vae.BN_STATS_IN_CONV = True
        assert bnstats_blocks(xd, m.block[0].weight, 2, kind == "dec") > 0
        assert any("bnstats" in t for t in tr.lines) == fused, tr.lines
        assert any(t.startswith("bn_apply_part") for t in tr.lines) == fused, tr.lines
        runs.append((y.detach(), xd.grad, {k: p.grad for k, p in m.named_parameters()},
                     {k: v.clone() for k, v in m.state_dict().items()}, gy))
    (y1, g1, p1, s1, gy), (y2, g2, p2, s2, _) = runs

    def rel(a, r):
        return float((a.double() - r.double()).abs().max() / r.double().abs().max().clamp_min(1e-30))
    # against the separate conv + BN launches: the same formulas, fp64 sums in another order
    assert rel(y1, y2) < 1e-5
    assert rel(g1, g2) < 1e-5
    for k in p1:
        assert rel(p1[k], p2[k]) < 1e-5, k
    for k in s1:
        if s1[k].is_floating_point():
            assert rel(s1[k], s2[k]) < 1e-6, k
        else:
            assert torch.equal(s1[k], s2[k]), k
    # against torch fp64 (north_star: 1e-4 relative)
    yr, rm, rv = _ref(kind, m0, x.double())
    assert rel(y1.cpu(), yr) < 1e-4
    assert rel(s1["block.1.running_mean"].cpu(), rm) < 1e-5
    assert rel(s1["block.1.running_var"].cpu(), rv) < 1e-5
