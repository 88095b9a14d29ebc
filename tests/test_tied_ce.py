"""The fused tied-logits masked cross-entropy of the priors' training loss (csrc/tvq_ce.hip,
bidirectional_transformer._TiedCE) against torch on the CPU: F.cross_entropy over the masked
rows of embed @ W[:K]^T + bias[:, :K] (bidirectional_transformer.py:186-191,
maskgit.py:183-191) -- the loss and the gradients of embed, the tied table and the bias --
at the bench's LF (6400 rows, D 128, n 24) and HF (24576 rows, D 32, n 96) shapes and at odd
sizes; every backward run twice must be bitwise equal.  Tolerance: loss rel 1e-5, gradients
rel-L2 1e-5 (fp32 reassociation)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).norm() / (b.norm() + 1e-30))


@pytest.mark.parametrize("B,n,D,K", [(256, 24, 128, 512), (256, 96, 32, 512), (7, 13, 64, 96),
                                     (3, 40, 32, 32)])
def test_tied_ce_vs_torch(B, n, D, K, cuda):
    from timevqvae.hip._native import plan_trace
    from timevqvae.models.bidirectional_transformer import _TiedCE
    gen = torch.Generator().manual_seed(B * n + D + K)
    h = torch.randn(B, n, D, generator=gen)
    W = torch.randn(K + 1, D, generator=gen) * D ** -0.5
    bias = torch.randn(n, K + 1, generator=gen) * 0.1
    target = torch.randint(0, K, (B, n), generator=gen)
    keep = torch.rand(B, n, generator=gen) < 0.4
    hc, Wc, bc = (t.clone().requires_grad_(True) for t in (h, W, bias))
    logits = (hc @ Wc.t() + bc)[:, :, :-1]
    lc = F.cross_entropy(logits[~keep], target[~keep])
    lc.backward()
    grads = []
    for _ in range(2):
        hd, Wd, bd = (t.to(cuda).requires_grad_(True) for t in (h, W, bias))
        with plan_trace() as tr:
            ld = _TiedCE.apply(hd, Wd, bd, K, target.to(cuda), keep.to(cuda))
            ld.backward()
            torch.cuda.synchronize()
        assert tr.has("tied_ce_fwd") and tr.has("tied_ce_bwd"), tr.lines
        grads.append((float(ld), hd.grad.cpu(), Wd.grad.cpu(), bd.grad.cpu()))
    assert grads[0][0] == grads[1][0]
    for a, b in zip(grads[0][1:], grads[1][1:]):
        assert torch.equal(a, b)
    v, dh, dW, db = grads[0]
    assert abs(v - float(lc)) <= 1e-5 * abs(float(lc)), (v, float(lc))
    assert rel(dh, hc.grad) < 1e-5, rel(dh, hc.grad)
    assert rel(dW, Wc.grad) < 1e-5, rel(dW, Wc.grad)
    assert rel(db, bc.grad) < 1e-5, rel(db, bc.grad)
    assert float(dW[K].abs().max()) == 0.0 and float(db[:, K].abs().max()) == 0.0


def test_maskgit_fused_ce_matches_unfused(cuda, monkeypatch):
    """MaskGIT.forward with TVQ_FUSED_CE (the fused loss; off by default) gives the unfused
    path's loss and transformer gradients on the same draws."""
    from test_stage2_golden import _maskgit
    from timevqvae.hip._native import plan_trace
    from timevqvae.models import maskgit as mgmod
    torch.manual_seed(0)
    x = torch.randn(4, 6, 128, device=cuda)
    y = torch.randint(0, 5, (4, 1), device=cuda)
    draws = {"ratio_l": [0.1, 0.5, 0.7, 0.3], "rand_l": torch.rand(4, 24), "ratio_h": [0.9, 0.2, 0.4, 0.6],
             "rand_h": torch.rand(4, 96), "cls_l": torch.rand(4, 1), "cls_h": torch.rand(4, 1)}
    res = []
    for fused in (False, True):
        monkeypatch.setattr(mgmod, "FUSED_CE", fused)
        mg = _maskgit(cuda).train()
        with plan_trace() as tr:
            loss, _ = mg(x, y, draws=draws)
            loss.backward()
            torch.cuda.synchronize()
        assert (len(tr.has("tied_ce_fwd")) == 2) == fused, tr.lines
        res.append((float(loss), {k: p.grad.clone() for k, p in mg.named_parameters()
                                  if p.grad is not None}))
    assert abs(res[0][0] - res[1][0]) <= 1e-5 * abs(res[0][0])
    for k, g in res[0][1].items():
        assert rel(res[1][1][k], g) < 1e-5, k
