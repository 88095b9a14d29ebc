"""The fused feed-forward branch of the LF prior (csrc/tvq_ffn.hip, hip.xf.fused_ff) against
the per-op HIP path it replaces (Linear+GELU, dropout, Linear+gate+residual; x-transformers
FeedForward in the pre-norm residual, bidirectional_transformer.py:92-110) and against torch
fp32: output, input / residual gradients and every weight and bias gradient, at the bench's
6400 token rows and at a ragged row count, with dropout 0.3 (the same device masks) and
with the layer-dropout gate.  Tolerance: rel-L2 1e-5 (fp32, MFMA summation order)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).norm() / (b.norm() + 1e-30))


def _run(ff, x, r, gate, fused, gy):
    from timevqvae.hip import rng, xf
    from timevqvae.hip._native import plan_trace
    rng.manual_seed(3)
    xf.FUSED_FF = fused
    try:
        xx, rr = x.clone().requires_grad_(True), r.clone().requires_grad_(True)
        for p in ff.parameters():
            p.grad = None
        with plan_trace() as tr:
            y = ff(xx, rr, gate)
            y.backward(gy)
            torch.cuda.synchronize()
    finally:
        xf.FUSED_FF = True
    assert bool(tr.has("ffn_fwd")) == fused and bool(tr.has("ffn_bwd")) == fused, tr.lines
    return y.detach(), xx.grad, rr.grad, {k: p.grad.clone() for k, p in ff.named_parameters()}


@pytest.mark.parametrize("B,n,p,gated", [(256, 25, 0.3, True), (256, 25, 0.0, False),
                                          (7, 13, 0.3, False)])
def test_fused_ff_matches_per_op_path(B, n, p, gated, cuda):
    from timevqvae.models.bidirectional_transformer import FeedForward
    torch.manual_seed(B + n)
    ff = FeedForward(128, 1, p).to(cuda).train()
    x = torch.randn(B, n, 128, device=cuda)
    r = torch.randn(B, n, 128, device=cuda)
    gy = torch.randn(B, n, 128, device=cuda)
    gate = torch.ones(1, device=cuda) if gated else None
    a = _run(ff, x, r, gate, True, gy)
    b = _run(ff, x, r, gate, False, gy)
    for u, v, what in zip(a[:3], b[:3], ("y", "dx", "dr")):
        assert rel(u, v) < 1e-5, (what, rel(u, v))
    for k in b[3]:
        assert rel(a[3][k], b[3][k]) < 1e-5, (k, rel(a[3][k], b[3][k]))
    if p == 0.0:  # and against torch's own FeedForward arithmetic
        xx = x.clone().requires_grad_(True)
        l1, l2 = ff.ff[0][0], ff.ff[2]
        want = r + F.linear(F.gelu(F.linear(xx, l1.weight, l1.bias)), l2.weight, l2.bias)
        assert rel(a[0], want) < 1e-5


def test_fused_ff_gate_zero_drops_the_branch(cuda):
    """gate 0 (a dropped branch under graph capture): y == r, no gradient reaches x, and
    every weight / bias gradient of the branch is exactly zero (dW2 / db2 come from
    gate * gy, so a dropped forward adds nothing under gradient accumulation either)."""
    from timevqvae.models.bidirectional_transformer import FeedForward
    torch.manual_seed(1)
    ff = FeedForward(128, 1, 0.3).to(cuda).train()
    x = torch.randn(64, 25, 128, device=cuda)
    r = torch.randn(64, 25, 128, device=cuda)
    gy = torch.randn(64, 25, 128, device=cuda)
    y, dx, dr, grads = _run(ff, x, r, torch.zeros(1, device=cuda), True, gy)
    assert torch.equal(y, r)
    assert float(dx.abs().max()) == 0.0 and torch.equal(dr, gy)
    for k, g in grads.items():
        assert float(g.abs().max()) == 0.0, k
    # and the per-op path agrees
    _, _, _, ref = _run(ff, x, r, torch.zeros(1, device=cuda), False, gy)
    for k, g in ref.items():
        assert float(g.abs().max()) == 0.0, k
