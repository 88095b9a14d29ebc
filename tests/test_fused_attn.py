"""The fused attention branch of the LF prior (csrc/tvq_xattn.hip, hip.xf.attn_branch) against
the per-op HIP path it replaces (RMSNorm with the residual output, the QKV GEMM, attention with
dropout, the gated out-projection Linear; x-transformers pre-norm attention layer,
bidirectional_transformer.py:92-110) and against torch fp32: output, input gradient and every
weight / gain gradient, at the bench's 256 sequences of 25 tokens and at ragged shapes, with
attention dropout 0.3 (the same device masks) and with the layer-dropout gate.
Tolerance: rel-L2 1e-5 (fp32, MFMA summation order)."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).norm() / (b.norm() + 1e-30))


def _layer(p, seed):
    from timevqvae.models.bidirectional_transformer import Attention, RMSNorm
    torch.manual_seed(seed)
    norm, attn = RMSNorm(128), Attention(128, 2, 64, p)
    with torch.no_grad():
        norm.g.uniform_(0.5, 1.5)
    return norm.cuda(), attn.cuda().train()


def _run(norm, attn, x, gate, fused, gy, p):
    from timevqvae.hip import rng, xf
    from timevqvae.hip._native import plan_trace
    rng.manual_seed(3)
    rng._calls[0] = 0
    xx = x.clone().requires_grad_(True)
    for m in (norm, attn):
        for q in m.parameters():
            q.grad = None
    with plan_trace() as tr:
        if fused:
            assert xf.attn_branch_supported(xx, norm.g, attn)
            y = xf.attn_branch(xx, norm.g, attn, gate, p)
        else:
            n, r = xf.rmsnorm_res(xx, norm.g)
            y = attn(n, residual=r, gate=gate)
        y.backward(gy)
        torch.cuda.synchronize()
    assert bool(tr.has("attn_branch_fwd")) == fused and bool(tr.has("attn_branch_bwd")) == fused
    grads = {"x": xx.grad, "g": norm.g.grad}
    grads.update({k: q.grad.clone() for k, q in attn.named_parameters()})
    return y.detach(), grads


@pytest.mark.parametrize("B,n,p,gated", [(256, 25, 0.3, True), (256, 25, 0.0, False),
                                          (7, 13, 0.3, False), (3, 32, 0.0, True), (5, 1, 0.0, False)])
def test_fused_attn_matches_per_op_path(B, n, p, gated, cuda):
    norm, attn = _layer(p, B + n)
    x = torch.randn(B, n, 128, device=cuda)
    gy = torch.randn(B, n, 128, device=cuda)
    gate = torch.ones(1, device=cuda) if gated else None
    ya, ga = _run(norm, attn, x, gate, True, gy, p)
    yb, gb = _run(norm, attn, x, gate, False, gy, p)
    assert rel(ya, yb) < 1e-5, rel(ya, yb)
    for k in gb:
        if n == 1 and k in ("to_q.weight", "to_k.weight"):
            # one token: softmax over one key is exactly 1, the true dQ / dK are 0 and both
            # paths hold rounding noise only
            scale = float(gb["to_v.weight"].abs().max())
            assert float((ga[k] - gb[k]).abs().max()) <= 1e-5 * scale, k
            continue
        assert rel(ga[k], gb[k]) < 1e-5, (k, rel(ga[k], gb[k]))
    if p == 0.0:  # and against torch's own arithmetic of the layer
        xx = x.clone()
        xn = F.normalize(xx, dim=-1) * math.sqrt(128) * norm.g
        q, k, v = (F.linear(xn, w).view(B, n, 2, 64).transpose(1, 2)
                   for w in (attn.to_q.weight, attn.to_k.weight, attn.to_v.weight))
        o = torch.softmax(q @ k.transpose(-1, -2) / 8.0, -1) @ v
        want = xx + F.linear(o.transpose(1, 2).reshape(B, n, 128), attn.to_out.weight)
        assert rel(ya, want) < 1e-5, rel(ya, want)


def test_fused_attn_gate_zero_drops_the_branch(cuda):
    """gate 0 (a dropped branch under graph capture): y == x, dx == gy, and the out-projection
    gets an exactly-zero gradient (dWo from gate * gy)."""
    norm, attn = _layer(0.3, 1)
    x = torch.randn(64, 25, 128, device=cuda)
    gy = torch.randn(64, 25, 128, device=cuda)
    y, g = _run(norm, attn, x, torch.zeros(1, device=cuda), True, gy, 0.3)
    assert torch.equal(y, x)
    assert torch.equal(g["x"], gy)
    for k in ("to_out.weight", "to_q.weight", "to_k.weight", "to_v.weight", "g"):
        assert float(g[k].abs().max()) == 0.0, k
