"""MaskGIT sampling on the HIP path vs the oracle.

The reference draws with torch's RNG (Categorical.sample, uniform_ Gumbel noise), which a
GPU kernel cannot reproduce; the oracle's `sample_step` restates one decoding step of
first_pass / second_pass (maskgit.py:294-411) with the noise injected, and the kernels are
run on the same injected noise.  Parity: sampled codes and re-masked token sets exact.
"""
import os
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

pytestmark = pytest.mark.gpu


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
    u_cat = torch.rand(B, n, generator=g)
    u_g = torch.rand(B, n, generator=g)
    ref = O.sample_step(logits, s, mask_id, t, T, torch.full((B,), n), temp, u_cat, u_g)

    ratio = (t + 1) / T
    sampled, selp = maskgit_sample(logits.to(cuda), s.to(cuda), mask_id, u_cat=u_cat.to(cuda))
    k = mask_len(n, O.gamma_cosine(ratio))
    out = maskgit_remask(selp, k, temp * (1.0 - ratio), sampled, mask_id, u_gumbel=u_g.to(cuda))
    torch.cuda.synchronize()
    # categorical draw: exact vs the double-precision inverse CDF
    probs = torch.softmax(logits.double(), -1)
    cdf = torch.cumsum(probs, -1)
    want = torch.searchsorted(cdf, u_cat.double().unsqueeze(-1) * cdf[..., -1:],
                              right=True).squeeze(-1)
    want = torch.where(s == mask_id, want.clamp(max=K - 1), s)
    assert torch.equal(sampled.cpu(), want)
    assert torch.equal(out.cpu(), ref)
    assert int((out == mask_id).sum(1).max()) == k == int((out == mask_id).sum(1).min())


def test_sample_never_draws_zero_probability_code(cuda):
    """u = 0 with leading codes whose probability underflows to 0: the draw is the first
    code of positive probability (torch's Categorical never samples a 0-probability code)."""
    from timevqvae.hip.sample import maskgit_sample
    K = 512
    logits = torch.zeros(2, 3, K)
    logits[..., :70] = -1e4  # exp underflows: p = 0 for codes 0..69 (two lanes' chunks)
    s = torch.full((2, 3), K, dtype=torch.int64)
    u = torch.zeros(2, 3)
    sampled, selp = maskgit_sample(logits.to(cuda), s.to(cuda), K, u_cat=u.to(cuda))
    assert (sampled.cpu() == 70).all()
    assert (selp.cpu() > 0).all()


def test_sample_u_near_one_never_draws_trailing_zero_probability_code(cuda):
    """u just below 1 with trailing codes of probability 0: no prefix may exceed v after
    rounding, and the fallback must still land on a positive-probability code (the last
    one), never the zero-probability tail."""
    from timevqvae.hip.sample import maskgit_sample
    K = 512
    logits = torch.zeros(2, 3, K)
    logits[..., 300:] = -1e4  # p = 0 for codes 300..511 (the last 26 lanes' chunks)
    s = torch.full((2, 3), K, dtype=torch.int64)
    for u0 in (1.0 - 2.0 ** -24, 1.0 - 2.0 ** -20, 0.999999):
        u = torch.full((2, 3), u0)
        sampled, selp = maskgit_sample(logits.to(cuda), s.to(cuda), K, u_cat=u.to(cuda))
        assert (sampled.cpu() < 300).all() and (sampled.cpu() >= 290).all(), sampled
        assert (selp.cpu() > 0).all()


def test_mask_by_random_topk_exact_k(cuda):
    """mask_by_random_topk keeps exactly mask_len per row; known tokens (+inf) never mask."""
    from timevqvae.hip.sample import maskgit_remask
    g = torch.Generator().manual_seed(2)
    p = torch.rand(64, 40, generator=g)
    p[:, :10] = float("inf")
    m = maskgit_remask(p.to(cuda), 17, 2.0, want_masking=True)
    torch.cuda.synchronize()
    assert m.sum(1).eq(17).all() and not m[:, :10].any()


def test_codebook_gather_nchw(cuda):
    from timevqvae.hip.sample import codebook_gather_nchw
    g = torch.Generator().manual_seed(3)
    E = torch.randn(50, 16, generator=g)
    s = torch.randint(0, 50, (5, 3 * 8), generator=g)
    out = codebook_gather_nchw(s.to(cuda), E.to(cuda), 3, 8)
    want = E[s].transpose(1, 2).reshape(5, 16, 3, 8)
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
