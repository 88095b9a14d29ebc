"""The priors' training forward with the Linears that meet without a nonlinearity folded:
Upscale's last Conv1d into the HF prior's project_in (hip.upscale.hf_embed_folded: a 256 -> 32
conv with W_l W2 instead of 256 -> 128 then the (B, m + 1, 256) embedding through the 256 -> 32
Linear) and project_out into pred_head's Linear (hip.linear.weight_product, both priors;
reference bidirectional_transformer.py:12-30,166-236), against the unfolded chains of this
library and against torch fp64 autograd of the reference formula.  The two chains sum in another order (fp32 reassociation), so the bars
are relative fp32 tolerances, written per check."""
import copy
import random

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _prior(cuda, dropout, kind="hf"):
    from timevqvae.hip import rng
    from timevqvae.models import BidirectionalTransformer
    rng.manual_seed(11)
    torch.manual_seed(3)
    if kind == "hf":  # config.yaml prior_model_h with the config-B token grid
        tf = BidirectionalTransformer("hf", 96, {"lf": 64, "hf": 64}, 128, hidden_dim=32,
                                      n_layers=1, heads=1, ff_mult=1, use_rmsnorm=True,
                                      p_unconditional=0.2, n_classes=5, model_dropout=dropout,
                                      emb_dropout=dropout, num_tokens_l=24)
    else:  # prior_model_l
        tf = BidirectionalTransformer("lf", 24, {"lf": 64, "hf": 64}, 128, hidden_dim=128,
                                      n_layers=4, heads=2, ff_mult=1, use_rmsnorm=True,
                                      p_unconditional=0.2, n_classes=5, model_dropout=dropout,
                                      emb_dropout=dropout)
    tf = tf.to(cuda).train()
    with torch.no_grad():
        for p in tf.parameters():
            if p.dim() == 1 and p.shape[0] > 1:
                p.normal_(0.0, 0.2)
        tf.pos_emb.weight.normal_()
        tf.class_condition_emb.weight.normal_()
        tf.bias.normal_(0.0, 0.1)
    return tf


def _run(tf, sl, sh, y, gy, fold, class_rand, monkeypatch):
    from timevqvae.hip import rng
    from timevqvae.models import bidirectional_transformer as bt
    rng.manual_seed(11)
    random.seed(11)  # host-side layer-dropout decisions
    torch.manual_seed(11)
    tf._class_rand = class_rand
    used = []
    inner = bt.hf_embed_folded
    monkeypatch.setattr(bt, "hf_embed_folded", lambda *a: used.append(1) or inner(*a))
    monkeypatch.setattr(bt, "HF_EMBED_FOLD", fold)
    monkeypatch.setattr(bt, "HEAD_FOLD", fold)
    out = tf(sl, sh, y) if sh is not None else tf(sl, class_condition=y)
    out.backward(gy)
    torch.cuda.synchronize()
    monkeypatch.undo()
    return (out.detach(), {k: None if p.grad is None else p.grad.clone()
                          for k, p in tf.named_parameters()}, len(used))


def _rel(a, r):
    return float((a.double() - r.double()).abs().max() / r.double().abs().max().clamp_min(1e-30))


@pytest.mark.parametrize("kind,B,dropout", [("hf", 256, 0.0), ("hf", 256, 0.3), ("hf", 7, 0.3),
                                             ("lf", 256, 0.3), ("lf", 5, 0.0)])
def test_prior_folds_equal_unfolded(kind, B, dropout, cuda, monkeypatch):
    """Logits, every parameter gradient and the BatchNorm running statistics of the folded
    training forward+backward against the unfolded one (the same dropout masks: the same
    draw sites in the same order)."""
    tf = _prior(cuda, dropout, kind)
    tf2 = copy.deepcopy(tf)
    g = torch.Generator().manual_seed(B)
    sl = torch.randint(0, 65, (B, 24), generator=g).to(cuda)
    sh = torch.randint(0, 65, (B, 96), generator=g).to(cuda) if kind == "hf" else None
    y = torch.randint(0, 5, (B, 1), generator=g).to(cuda)
    u = torch.rand(B, generator=g)
    gy = torch.randn(B, 96 if kind == "hf" else 24, 64, generator=g).to(cuda)
    o1, p1, n1 = _run(tf, sl, sh, y, gy, True, u, monkeypatch)
    o2, p2, n2 = _run(tf2, sl, sh, y, gy, False, u, monkeypatch)
    assert (n1, n2) == ((1, 0) if kind == "hf" else (0, 0))
    assert _rel(o1, o2) < 2e-5
    for k in p1:
        assert (p1[k] is None) == (p2[k] is None), k
        if p1[k] is not None:
            assert _rel(p1[k], p2[k]) < 1e-4, k
    s1, s2 = tf.state_dict(), tf2.state_dict()
    for k in s1:
        if s1[k].is_floating_point():
            assert _rel(s1[k], s2[k]) < 1e-5, k


def test_hf_embed_folded_op_vs_torch_fp64(cuda):
    """The folded op alone against torch fp64 autograd of project_in(cat(cls, cat(conv(x)^T, th)
    + pos[:m])): output and the gradients of all seven inputs (parameters returned, no flat
    gradient sinks)."""
    from timevqvae.hip.upscale import hf_embed_folded, hf_embed_supported
    torch.manual_seed(5)
    B, H, m, D, d = 64, 256, 96, 128, 32
    x = torch.randn(B, H, m)
    th = torch.randn(B, m, D)
    cls = torch.randn(B, 1, 2 * D)
    W_in = torch.randn(d, 2 * D) / (2 * D) ** 0.5
    W2 = torch.randn(D, H, 3) / (3 * H) ** 0.5
    b2 = torch.randn(D) * 0.1
    pos = torch.randn(97, 2 * D)
    ins = [x, th, cls, W_in, W2, b2, pos]
    dv = [t.to(cuda).requires_grad_(True) for t in ins]
    rf = [t.double().requires_grad_(True) for t in ins]
    assert hf_embed_supported(dv[0], dv[1], dv[3], dv[4], dv[6])
    z = hf_embed_folded(*dv)
    up = F.conv1d(rf[0], rf[4], rf[5], padding=1).transpose(1, 2)
    emb = torch.cat([rf[2], torch.cat([up, rf[1]], -1) + rf[6][:m]], 1)
    zr = emb @ rf[3].t()
    gz = torch.randn(B, m + 1, d, dtype=torch.float64)
    z.backward(gz.float().to(cuda))
    zr.backward(gz)
    torch.cuda.synchronize()
    assert _rel(z.detach().cpu(), zr.detach()) < 1e-5
    for a, r, name in zip(dv, rf, ["x", "th", "cls", "W_in", "W2", "b2", "pos"]):
        assert _rel(a.grad.cpu(), r.grad) < 2e-5, name


def test_weight_product_vs_torch(cuda):
    """hip.linear.weight_product: W1 W2 and both gradients (no sinks) against torch fp64."""
    from timevqvae.hip.linear import weight_product
    torch.manual_seed(2)
    w1, w2 = torch.randn(128, 256), torch.randn(256, 32)
    a1, a2 = w1.to(cuda).requires_grad_(True), w2.to(cuda).requires_grad_(True)
    r1, r2 = w1.double().requires_grad_(True), w2.double().requires_grad_(True)
    g = torch.randn(128, 32, dtype=torch.float64)
    y = weight_product(a1, a2)
    y.backward(g.float().to(cuda))
    (r1 @ r2).backward(g)
    torch.cuda.synchronize()
    assert _rel(y.detach().cpu(), (r1 @ r2).detach()) < 1e-5
    assert _rel(a1.grad.cpu(), r1.grad) < 1e-5
    assert _rel(a2.grad.cpu(), r2.grad) < 1e-5
