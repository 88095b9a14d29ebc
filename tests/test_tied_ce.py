"""The priors' fused training loss head (bidirectional_transformer.tied_logits_ce,
tvq_tied_logits_ce: tied logits + masked cross-entropy + dlogits + dh in one pass;
reference bidirectional_transformer.py:186-191, maskgit.py:183-191) against (a) this
library's unfused chain (_TiedLogits -> masked_cross_entropy -> backward with the same root
gradient) and (b) torch fp64 autograd of the reference formula.  fp32 sums in another order:
relative tolerances written per check."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _rel(a, r):
    return float((a.double() - r.double()).abs().max() / r.double().abs().max().clamp_min(1e-30))


def _case(B, n, K, seed, cuda, frac=0.36):
    g = torch.Generator().manual_seed(seed)
    h = torch.randn(B, n, 128, generator=g)
    W = torch.randn(K + 1, 128, generator=g) / 128 ** 0.5 * 3
    bias = torch.randn(n, K + 1, generator=g) * 0.2
    tgt = torch.randint(0, K, (B, n), generator=g)
    keep = torch.rand(B, n, generator=g) >= frac
    keep[0, 0] = False  # at least one masked token
    return h, W, bias, tgt, keep


@pytest.mark.parametrize("B,n,K", [(256, 96, 512), (256, 24, 512), (7, 24, 64), (3, 97, 128)])
def test_tied_ce_vs_unfused_and_fp64(B, n, K, cuda, monkeypatch):
    from timevqvae.hip import linear
    from timevqvae.models.bidirectional_transformer import _TiedLogits, tied_logits_ce
    from timevqvae.hip.xf import masked_cross_entropy
    rescales = []
    inner = linear.scale_by
    monkeypatch.setattr(linear, "scale_by", lambda *a: rescales.append(1) or inner(*a))
    h, W, bias, tgt, keep = _case(B, n, K, B * n + K, cuda)
    one = torch.ones((), device=cuda)
    runs = []
    for fused in (True, False):
        hd = h.to(cuda).requires_grad_(True)
        Wd = W.to(cuda).requires_grad_(True)
        bd = bias.to(cuda).requires_grad_(True)
        if fused:
            loss = tied_logits_ce(hd, Wd, bd, K, tgt.to(cuda), keep.to(cuda), one)
        else:
            loss = masked_cross_entropy(_TiedLogits.apply(hd, Wd, bd, K), tgt.to(cuda), keep.to(cuda))
        torch.autograd.backward(loss, one)
        torch.cuda.synchronize()
        runs.append((loss.detach().cpu(), hd.grad.cpu(), Wd.grad.cpu(), bd.grad.cpu()))
    (l1, gh1, gW1, gb1), (l2, gh2, gW2, gb2) = runs
    assert not rescales  # the root gradient reached the backward as the forward's tensor
    assert _rel(l1, l2) < 1e-6
    assert _rel(gh1, gh2) < 1e-5
    assert _rel(gW1, gW2) < 1e-5
    assert _rel(gb1, gb2) < 1e-5
    assert torch.equal(gW1[K:], torch.zeros_like(gW1[K:]))  # the mask-token row
    # torch fp64 of the reference formula
    hr = h.double().requires_grad_(True)
    Wr = W.double().requires_grad_(True)
    br = bias.double().requires_grad_(True)
    logits = hr @ Wr[:K].t() + br[:, :K]
    lr = F.cross_entropy(logits[~keep], tgt[~keep])
    lr.backward()
    assert _rel(l1, lr.detach()) < 1e-5
    assert _rel(gh1, hr.grad) < 1e-4
    assert _rel(gW1, Wr.grad) < 1e-4
    assert _rel(gb1, br.grad) < 1e-4


def test_tied_ce_other_root_gradient(cuda):
    """A root gradient other than the `gscale` tensor the forward used scales every gradient
    (the rescale path; forward_backward passes the same tensor)."""
    from timevqvae.models.bidirectional_transformer import tied_logits_ce
    h, W, bias, tgt, keep = _case(4, 24, 64, 5, cuda)
    one = torch.ones((), device=cuda)
    grads = []
    for root in (one, torch.full((), 2.5, device=cuda)):
        hd = h.to(cuda).requires_grad_(True)
        Wd = W.to(cuda).requires_grad_(True)
        bd = bias.to(cuda).requires_grad_(True)
        loss = tied_logits_ce(hd, Wd, bd, 64, tgt.to(cuda), keep.to(cuda), one)
        torch.autograd.backward(loss, root)
        torch.cuda.synchronize()
        grads.append((hd.grad.cpu(), Wd.grad.cpu(), bd.grad.cpu()))
    for a, b in zip(grads[1], grads[0]):
        assert _rel(a, 2.5 * b) < 1e-6
