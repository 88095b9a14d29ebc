"""MaskGIT sampling on the HIP path vs the oracle.

The reference draws with torch's RNG (Categorical.sample -> multinomial's exponential race,
uniform_ Gumbel noise), which a GPU kernel cannot reproduce; the oracle restates one decoding
step of first_pass / second_pass (maskgit.py:294-411) with the noise injected
(race_sample: argmax of logits + Gumbel; remask_step), and the kernels are run on the same
injected noise.  Parity: sampled codes and re-masked token sets exact; p(sampled) within
2e-6 relative of the double softmax.  The device noise itself is checked for the
distribution it draws (frequencies) and for never drawing a 0-probability code.
"""
import os
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

pytestmark = pytest.mark.gpu


def _gumbel(shape, g):
    u = torch.rand(shape, generator=g).clamp(1e-7, 1 - 1e-7)
    return -torch.log(-torch.log(u))


@pytest.mark.parametrize("B,n,K,t,T,temp", [(16, 96, 512, 0, 1, 4.0), (32, 24, 512, 3, 10, 10.0),
                                             (8, 24, 64, 9, 10, 10.0), (4, 7, 33, 0, 3, 1.0)])
def test_sample_step_vs_oracle(B, n, K, t, T, temp, cuda):
    from oracle import tvq_oracle as O
    from timevqvae.hip.sample import mask_len, maskgit_remask, maskgit_sample
    g = torch.Generator().manual_seed(11 + t)
    logits = 3.0 * torch.randn(B, n, K, generator=g)
    mask_id = K
    s = torch.randint(0, K, (B, n), generator=g)
    n_known = n - int(np.floor(n * O.gamma_cosine(t / T))) if t > 0 else 0
    for i in range(B):  # the first n_known positions of a random order are already decoded
        perm = torch.randperm(n, generator=g)
        s[i, perm[n_known:]] = mask_id
    gum = _gumbel((B, n, K), g)
    u_g = torch.rand(B, n, generator=g)

    ratio = (t + 1) / T
    sampled, selp = maskgit_sample(logits.to(cuda), s.to(cuda), mask_id, gumbel=gum.to(cuda))
    k = mask_len(n, O.gamma_cosine(ratio))
    out = maskgit_remask(selp, k, temp * (1.0 - ratio), sampled, mask_id, u_gumbel=u_g.to(cuda))
    torch.cuda.synchronize()
    # the race draw: exact (same fp32 keys, first index of the maximum)
    want, sel = O.race_sample(logits, s, mask_id, gum)
    assert torch.equal(sampled.cpu(), want)
    # p(sampled): the fp32 softmax within 2e-6 relative of the double one
    known = s != mask_id
    assert torch.isinf(selp.cpu()[known]).all()
    got = selp.cpu()[~known].double()
    assert float(((got - sel[~known]).abs() / sel[~known]).max()) < 2e-6
    # the re-mask on the kernel's p(sampled): exact
    ref = O.remask_step(selp.cpu(), sampled.cpu(), mask_id, t, T, torch.full((B,), n), temp, u_g)
    assert torch.equal(out.cpu(), ref)
    assert int((out == mask_id).sum(1).max()) == k == int((out == mask_id).sum(1).min())


def test_sample_never_draws_zero_probability_code(cuda):
    """Codes whose fp32 softmax probability is 0 (logit 1e4 below the max) are never drawn
    by the device noise (Gumbel within [-2.9, 17.4]), wherever they sit in the row -- torch's
    multinomial never samples a 0-probability code -- and the draws spread over the rest."""
    from timevqvae.hip import rng
    from timevqvae.hip.sample import maskgit_sample
    K = 512
    logits = torch.zeros(64, 96, K)
    logits[..., :70] = -1e4
    logits[..., 300:] = -1e4
    s = torch.full((64, 96), K, dtype=torch.int64)
    rng.manual_seed(3)
    sampled, selp = maskgit_sample(logits.to(cuda), s.to(cuda), K)
    sc = sampled.cpu()
    assert ((sc >= 70) & (sc < 300)).all()
    assert (selp.cpu() > 0).all()
    # uniform over the 230 live codes: every one drawn among 6144 draws, none > 3x its share
    counts = torch.bincount(sc.reshape(-1), minlength=K)[70:300]
    assert (counts > 0).all() and int(counts.max()) < 3 * 6144 / 230


def test_sample_race_frequencies(cuda):
    """The device-noise race draws Categorical(softmax(logits)): empirical frequencies over
    65536 draws of one 8-code distribution within 5 sigma of p."""
    from timevqvae.hip import rng
    from timevqvae.hip.sample import maskgit_sample
    K = 8
    lg = torch.tensor([0.0, 1.0, -1.0, 2.0, 0.5, -3.0, 1.5, 0.2])
    p = torch.softmax(lg.double(), 0)
    logits = lg.expand(256, 256, K).contiguous()
    s = torch.full((256, 256), K, dtype=torch.int64)
    rng.manual_seed(9)
    sampled, _ = maskgit_sample(logits.to(cuda), s.to(cuda), K)
    f = torch.bincount(sampled.cpu().reshape(-1), minlength=K).double() / 65536
    sig = (p * (1 - p) / 65536).sqrt()
    assert float(((f - p).abs() / sig).max()) < 5.0, (f, p)


@pytest.mark.parametrize("B,n,D,K", [(1024, 96, 128, 512), (5, 13, 128, 100), (3, 7, 64, 33)])
def test_tied_logits_sample_vs_oracle(B, n, D, K, cuda):
    """The fused head + draw (tvq_tied_logits_sample): its logits within 1e-5 of torch's
    h W[:K]^T + bias, its draw exactly the race on those logits, p(sampled) within 2e-6,
    known tokens kept; and the same draw as maskgit_sample on its logits."""
    from oracle import tvq_oracle as O
    from timevqvae.hip._native import plan_trace
    from timevqvae.hip.sample import maskgit_sample, tied_logits_sample
    g = torch.Generator().manual_seed(B + n + D + K)
    h = torch.randn(B, n, D, generator=g)
    W = torch.randn(K + 1, D, generator=g) * D ** -0.5
    bias = torch.randn(n, K + 1, generator=g) * 0.3
    mask_id = K
    s = torch.randint(0, K, (B, n), generator=g)
    s[torch.rand(B, n, generator=g) < 0.7] = mask_id
    gum = _gumbel((B, n, K), g)
    with plan_trace() as tr:
        sampled, selp, lg = tied_logits_sample(h.to(cuda), W.to(cuda), bias.to(cuda), K,
                                               s.to(cuda), mask_id, gumbel=gum.to(cuda),
                                               want_logits=True)
        torch.cuda.synchronize()
    assert tr.has("tied_logits_sample")
    want_l = (h.double() @ W[:K].double().t() + bias[:, :K].double()).float()
    lc = lg.cpu()
    assert float((lc - want_l).abs().max()) < 1e-5 * float(want_l.abs().max())
    want, sel = O.race_sample(lc, s, mask_id, gum)
    assert torch.equal(sampled.cpu(), want)
    known = s != mask_id
    assert torch.isinf(selp.cpu()[known]).all()
    got = selp.cpu()[~known].double()
    assert float(((got - sel[~known]).abs() / sel[~known]).max()) < 2e-6
    s2, p2 = maskgit_sample(lg, s.to(cuda), mask_id, gumbel=gum.to(cuda))
    assert torch.equal(s2.cpu(), sampled.cpu())
    assert float(((p2.cpu()[~known] - selp.cpu()[~known]).abs() / p2.cpu()[~known]).max()) < 2e-6


def test_tied_logits_sample_device_noise_matches_unfused(cuda):
    """With the device noise (no injection) the fused head draws exactly what maskgit_sample
    draws from the fused head's own logits at the same stream offset: both hash the same
    (stream key, token * K + code) counter."""
    from timevqvae.hip import rng
    from timevqvae.hip.sample import maskgit_sample, tied_logits_sample
    g = torch.Generator().manual_seed(77)
    B, n, D, K = 64, 96, 128, 512
    h = torch.randn(B, n, D, generator=g).to(cuda)
    W = (torch.randn(K + 1, D, generator=g) * D ** -0.5).to(cuda)
    bias = (torch.randn(n, K + 1, generator=g) * 0.3).to(cuda)
    s = torch.full((B, n), K, dtype=torch.int64, device=cuda)
    rng.manual_seed(4)
    a, pa, lg = tied_logits_sample(h, W, bias, K, s, K, site=7, want_logits=True)
    rng.manual_seed(4)
    b, pb = maskgit_sample(lg, s, K, site=7)
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    assert float(((pa - pb).abs() / pb).max()) < 2e-6


def test_hf_eval_head_folded_matches_forward_hf(cuda):
    """The HF prior's eval draw path (BidirectionalTransformer._head_hf_eval: project_in folded
    into Upscale's last conv and the token / position / class tables, project_out composed
    with pred_head's Linear) gives forward_hf's logits within 1e-5 relative (fp32
    reassociation), null and real class; and the draw equals the race on those logits."""
    from oracle import tvq_oracle as O
    from timevqvae.hip._native import plan_trace
    mg = _maskgit(cuda)
    tf = mg.transformer_h
    K = mg.mask_token_ids["hf"]
    g = torch.Generator().manual_seed(21)
    B = 6
    s_l = torch.randint(0, mg.mask_token_ids["lf"], (B, mg.num_tokens_l), generator=g).to(cuda)
    s_h = torch.randint(0, K + 1, (B, mg.num_tokens_h), generator=g).to(cuda)
    for cls in (None, torch.randint(0, 5, (B, 1), generator=g).to(cuda)):
        with torch.no_grad():
            want = tf(s_l, s_h, class_condition=cls)
            u = torch.rand(want.shape, generator=g).clamp(1e-7, 1 - 1e-7)
            gum = -torch.log(-torch.log(u))
            with plan_trace() as tr:
                sampled, selp, got = tf.sample(s_l, s_h, class_condition=cls, mask_id=K,
                                               gumbel=gum.to(cuda), want_logits=True)
                torch.cuda.synchronize()
        assert tr.has("tied_logits_sample")
        err = float((got - want).norm() / want.norm())
        assert err < 1e-5, err
        race, _ = O.race_sample(got.cpu(), s_h.cpu(), K, gum)
        assert torch.equal(sampled.cpu(), race)


def test_mask_by_random_topk_exact_k(cuda):
    """mask_by_random_topk keeps exactly mask_len per row; known tokens (+inf) never mask."""
    from timevqvae.hip.sample import maskgit_remask
    g = torch.Generator().manual_seed(2)
    p = torch.rand(64, 40, generator=g)
    p[:, :10] = float("inf")
    m = maskgit_remask(p.to(cuda), 17, 2.0, want_masking=True)
    torch.cuda.synchronize()
    assert m.sum(1).eq(17).all() and not m[:, :10].any()


@pytest.mark.parametrize("B,V,D,H,W", [(5, 50, 16, 3, 8), (7, 513, 128, 3, 32),
                                         (3, 513, 32, 1, 96), (2, 9, 5, 3, 43)])
def test_codebook_gather_nchw(B, V, D, H, W, cuda):
    """Bit-exact lookups at the decoders' (3 x 8 / 3 x 32 tokens, D 128) and the HF eval
    head's projected-table (D 32) shapes, and a ragged one (positions not a multiple of the
    64-position tile)."""
    from timevqvae.hip.sample import codebook_gather_nchw
    g = torch.Generator().manual_seed(3)
    E = torch.randn(V, D, generator=g)
    s = torch.randint(0, V, (B, H * W), generator=g)
    out = codebook_gather_nchw(s.to(cuda), E.to(cuda), H, W)
    want = E[s].transpose(1, 2).reshape(B, D, H, W)
    assert torch.equal(out.cpu(), want)


def _maskgit(cuda):
    import bench
    tr = bench.JointTrainer(cuda, 1, length=64, channels=3)
    return tr.s2.maskgit.eval()


def test_iterative_decoding(cuda):
    """maskgit.py:413-446: every token decoded, codes in range, HF after LF; reproducible
    under the same seed; class-conditional path runs."""
    from timevqvae.hip import rng
    mg = _maskgit(cuda)
    rng.manual_seed(5)
    s_l, s_h = mg.iterative_decoding(num=12, device=cuda)
    rng.manual_seed(5)
    s_l2, s_h2 = mg.iterative_decoding(num=12, device=cuda)
    torch.cuda.synchronize()
    K_l, K_h = mg.mask_token_ids["lf"], mg.mask_token_ids["hf"]
    assert s_l.shape == (12, mg.num_tokens_l) and s_h.shape == (12, mg.num_tokens_h)
    assert int(s_l.max()) < K_l and int(s_h.max()) < K_h and int(s_l.min()) >= 0
    assert torch.equal(s_l, s_l2) and torch.equal(s_h, s_h2)
    c_l, c_h = mg.iterative_decoding(num=5, device=cuda, class_index=2)
    assert int(c_l.max()) < K_l and int(c_h.max()) < K_h


def test_sample_utils_decode(cuda):
    """unconditional_sample: batches of iterative decoding + decode_token_ind_to_timeseries;
    the decoder output equals the decoder run on the torch-gathered latent."""
    from timevqvae.utils.sample_utils import unconditional_sample
    mg = _maskgit(cuda)
    x_l, x_h, x = unconditional_sample(mg, 10, cuda, batch_size=4)
    assert x_l.shape == (10, 3, 64) and torch.allclose(x, x_l + x_h)
    assert torch.isfinite(x).all()
    s = torch.randint(0, mg.mask_token_ids["lf"], (3, mg.num_tokens_l), device=cuda)
    xh, zq = mg.decode_token_ind_to_timeseries(s, "lf", return_representations=True)
    E = mg.vq_model_l._codebook.embed
    want = E[s].transpose(1, 2).reshape(zq.shape)
    assert torch.equal(zq, want)


@pytest.mark.gpu
def test_graphed_sampler_equals_eager(cuda):
    """A replay of the captured sampling batch equals the eager batch from the same device
    seed (decode + FidelityEnhancer included), and successive replays differ."""
    from timevqvae.hip import rng
    from timevqvae.models import FidelityEnhancer
    from timevqvae.utils.sample_utils import GraphedSampler
    mg = _maskgit(cuda)
    fe = FidelityEnhancer(64, 3, {"fidelity_enhancer": {"dim": 8, "dim_mults": [1, 2, 4, 8],
                                                        "resnet_block_groups": 4}}).to(cuda)
    gs = GraphedSampler(mg, 48, cuda, class_index=1, fidelity_enhancer=fe)
    rng.manual_seed(7)
    got = [t.clone() for t in gs.sample()]
    again = [t.clone() for t in gs.sample()]
    rng.manual_seed(7)
    with torch.no_grad():
        rng.advance(cuda)
        s_l, s_h = mg.iterative_decoding(num=48, device=cuda, class_index=1)
        x_l = mg.decode_token_ind_to_timeseries(s_l, "lf")
        x_h = mg.decode_token_ind_to_timeseries(s_h, "hf")
        want = [x_l, x_h, x_l + x_h, fe(x_l + x_h)]
    for g, w in zip(got, want):
        assert torch.equal(g, w)
    assert not torch.equal(again[2], got[2])
