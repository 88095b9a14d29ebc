"""The fused eval LF prior (csrc/tvq_prior_eval.hip, one launch per decoding step) against
the unfused HIP path of BidirectionalTransformer.forward_lf and against the oracle
restatement (oracle/tvq_oracle.transformer_forward; bidirectional_transformer.py:166-192,
x-transformers restated as T1).  Tolerance: logits within 1e-4 relative (fp32; the fused
kernel sums features in another order)."""
import math

import pytest
import torch

from oracle import tvq_oracle as O

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).norm() / b.norm())


def _prior(cuda, depth=4, K=512, n=24, seed=7):
    from timevqvae.models import BidirectionalTransformer
    m = BidirectionalTransformer("lf", n, {"lf": K, "hf": K}, 128, hidden_dim=128, n_layers=depth,
                                 heads=2, ff_mult=1, use_rmsnorm=True, p_unconditional=0.2,
                                 n_classes=5)
    gen = torch.Generator().manual_seed(seed)
    sd = {}
    for k, v in m.state_dict().items():
        if not v.is_floating_point():
            sd[k] = v
        elif k.endswith((".g", ".gamma")) or (k.startswith("pred_head.2") and k.endswith("weight")):
            sd[k] = 1.0 + 0.1 * torch.randn(v.shape, generator=gen)
        else:
            sd[k] = torch.randn(v.shape, generator=gen) * (
                0.5 / math.sqrt(max(v.shape[-1], 1)) if v.dim() > 1 else 0.1)
    m.load_state_dict(sd)
    return m.to(cuda).eval(), sd


@pytest.mark.parametrize("depth,K,n,B,cond", [(4, 512, 24, 64, False), (4, 512, 24, 37, True),
                                              (2, 64, 24, 16, False), (1, 100, 7, 9, True)])
def test_fused_prior_matches_unfused_and_oracle(depth, K, n, B, cond, cuda):
    from timevqvae.hip import xf
    m, sd = _prior(cuda, depth, K, n)
    gen = torch.Generator().manual_seed(11)
    s = torch.randint(0, K + 1, (B, n), generator=gen)  # mask id K included
    y = torch.randint(0, 5, (B, 1), generator=gen) if cond else None
    sg, yg = s.to(cuda), (y.to(cuda) if cond else None)
    with torch.no_grad():
        assert xf.prior_lf_eval_supported(m, sg)
        fused = m(sg, class_condition=yg)
        xf.PRIOR_FUSED = False
        try:
            unfused = m(sg, class_condition=yg)
        finally:
            xf.PRIOR_FUSED = True
    cls = y if cond else torch.full((B, 1), 5, dtype=torch.long)
    ref = O.transformer_forward(O.Ctx(False), sd, "lf", s, None, cls, K, 2, depth)
    assert fused.shape == unfused.shape == ref.shape == (B, n, K)
    assert rel(fused, unfused) < 1e-4, rel(fused, unfused)
    assert rel(fused, ref) < 1e-4, rel(fused, ref)
    assert float((fused.cpu() - ref).abs().max()) <= 1e-3 * float(ref.abs().max())
    # what MaskGIT's decoding consumes: the per-token argmax (greedy choice / confidence
    # ranking) agrees with the oracle's wherever the oracle's top-2 logit gap exceeds the
    # fp32 reassociation noise (1e-4 of the row's logit scale)
    top2 = torch.topk(ref.double(), 2, dim=-1).values
    gap = top2[..., 0] - top2[..., 1]
    scale = ref.double().abs().amax(-1)
    clear = gap > 1e-4 * scale
    agree = fused.cpu().argmax(-1) == ref.argmax(-1)
    assert bool(agree[clear].all()), int((~agree & clear).sum())
    assert float(clear.float().mean()) > 0.99


@pytest.mark.parametrize("depth,K,n,B,cond", [(4, 512, 24, 64, False), (2, 100, 7, 9, True)])
def test_fused_prior_draw(depth, K, n, B, cond, cuda):
    """tvq_prior_lf_eval_sample (the decoding step's draw in the prior's launch): its logits
    equal the logits-only launch's within 1e-6, its draw is exactly the oracle race on those
    logits with the injected Gumbel noise, p(sampled) within 2e-6 of the double softmax,
    known tokens kept; with the device noise it draws what maskgit_sample draws from the
    same logits at the same stream offset."""
    from timevqvae.hip import rng, xf
    from timevqvae.hip._native import plan_trace
    from timevqvae.hip.sample import maskgit_sample
    m, sd = _prior(cuda, depth, K, n)
    gen = torch.Generator().manual_seed(5)
    s = torch.randint(0, K, (B, n), generator=gen)
    s[torch.rand(B, n, generator=gen) < 0.6] = K  # mask id K: drawn; the rest kept
    y = torch.randint(0, 5, (B, 1), generator=gen) if cond else None
    sg, yg = s.to(cuda), (y.to(cuda) if cond else None)
    u = torch.rand(B, n, K, generator=gen).clamp(1e-7, 1 - 1e-7)
    gum = -torch.log(-torch.log(u))
    with torch.no_grad(), plan_trace() as tr:
        sampled, selp, lg = xf.prior_lf_eval_sample(m, sg, yg, K, gumbel=gum.to(cuda),
                                                    want_logits=True)
        plain = xf.prior_lf_eval(m, sg, yg)
        torch.cuda.synchronize()
    assert tr.has("prior_lf_eval_sample")
    assert float((lg - plain).abs().max()) <= 1e-6 * float(plain.abs().max())
    want, sel = O.race_sample(lg.cpu(), s, K, gum)
    assert torch.equal(sampled.cpu(), want)
    unk = s == K
    assert torch.isinf(selp.cpu()[~unk]).all()
    assert float(((selp.cpu()[unk].double() - sel[unk]).abs() / sel[unk]).max()) < 2e-6
    with torch.no_grad():
        rng.manual_seed(8)
        a, pa, lg2 = xf.prior_lf_eval_sample(m, sg, yg, K, site=3, want_logits=True)
        rng.manual_seed(8)
        b, pb = maskgit_sample(lg2, sg, K, site=3)
        torch.cuda.synchronize()
    assert torch.equal(a, b)
    fin = torch.isfinite(pb)
    assert float(((pa[fin] - pb[fin]).abs() / pb[fin]).max()) < 2e-6
    # the product form (no logits copy: the sampler's launch) draws the same codes with the
    # same p(sampled) bits
    with torch.no_grad():
        rng.manual_seed(8)
        c, pc = xf.prior_lf_eval_sample(m, sg, yg, K, site=3)
        torch.cuda.synchronize()
    assert torch.equal(c, a)
    assert torch.equal(pc, pa)


def test_fused_prior_declines_unaligned_weights(cuda):
    """tvq_prior_lf_eval reads weights with 16-byte loads: a parameter whose storage is not
    16-byte aligned (e.g. packed after an odd-sized one in a flat buffer) must send the
    prior down the unfused path, not raise (prior_lf_eval_supported)."""
    from timevqvae.hip import xf
    m, _ = _prior(cuda, 1, 64, 24)
    s = torch.randint(0, 65, (4, 24), device=cuda)
    w = m.blocks.project_in.weight
    buf = torch.empty(w.numel() + 1, device=cuda)
    buf[1:].copy_(w.detach().reshape(-1))
    with torch.no_grad():
        assert xf.prior_lf_eval_supported(m, s)
        w.data = buf[1:].view_as(w)  # 4 bytes past a 256-byte-aligned allocation
        assert not xf.prior_lf_eval_supported(m, s)
        m(s)  # the unfused path still runs


def test_fused_prior_not_used_when_training_or_grad(cuda):
    from timevqvae.hip import xf
    m, _ = _prior(cuda, 1, 64, 24)
    s = torch.randint(0, 65, (4, 24), device=cuda)
    assert not xf.prior_lf_eval_supported(m, s)  # parameters require grad, grad enabled
    with torch.no_grad():
        assert xf.prior_lf_eval_supported(m, s)
        m.train()
        assert not xf.prior_lf_eval_supported(m, s)
