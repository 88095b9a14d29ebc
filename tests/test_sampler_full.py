"""BASELINE configs[4] at its own size: MaskGIT iterative decoding + LF/HF decoding of 1024
trajectories with the configs/config.yaml architecture (T=256, C=6, K=512; LF prior 4
layers x 128 wide x 2 heads, HF prior 1 x 32 x 1 head) -- the bench's stage2 weights.

Reference: maskgit.py:294-477 (first_pass / second_pass / iterative_decoding /
decode_token_ind_to_timeseries), utils/sample_utils.py:5-64, generation/sampler.py:141-169.

Parity at full size:
  - every decoding step runs the product's draw (MaskGIT.sample_tokens: the LF prior's
    fused eval kernel + the race kernel; the HF prior's fused head + race, whose logits
    never reach memory, exported here for the check) with injected noise (Gumbel noise for
    the Categorical race, u_gumbel for the confidence noise); each step's logits equal the
    oracle transformer (oracle/tvq_oracle.transformer_forward) on the same tokens within
    1e-4 relative, the draws equal the oracle race (tvq_oracle.race_sample) on those
    logits exactly, p(sampled) is within 2e-6 of the double softmax, and the re-mask
    equals tvq_oracle.remask_step exactly;
  - the decoded series of a 64-row subset equal the oracle decoder within 1e-4 relative;
  - the graphed batch (GraphedSampler) equals the eager batch bit for bit, every token is
    decoded, codes are in range, and x == x_l + x_h.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

NUM = 1024


def rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).norm() / b.norm())


@pytest.fixture(scope="module")
def mg(cuda):
    import bench
    tr = bench.JointTrainer(cuda, 1)  # config.yaml architecture at T=256, C=6, K=512
    m = tr.s2.maskgit.eval()
    assert (m.num_tokens_l, m.num_tokens_h) == (24, 96)
    assert m.mask_token_ids == {"lf": 512, "hf": 512}
    return m


def _state(mod):
    return {k: v.detach().cpu() for k, v in mod.state_dict().items()}


def test_decode_1024_stepwise_vs_oracle(mg, cuda):
    from oracle import tvq_oracle as O
    from timevqvae.hip._native import plan_trace
    from timevqvae.hip.sample import mask_len, maskgit_remask
    g = torch.Generator().manual_seed(2024)
    pl = mg.config["MaskGIT"]["prior_model_l"]
    ph = mg.config["MaskGIT"]["prior_model_h"]
    sd_l, sd_h = _state(mg.transformer_l), _state(mg.transformer_h)
    null = torch.full((NUM, 1), mg.transformer_l.n_classes, dtype=torch.long)
    ctx = O.Ctx(False)

    def drive(kind, s, T, temp, n0, draw_fn, ref_fn):
        K = mg.mask_token_ids[kind]
        for t in range(T):
            u = torch.rand(NUM, n0, K, generator=g).clamp(1e-7, 1 - 1e-7)
            gum = -torch.log(-torch.log(u))
            del u
            # the product's draw (MaskGIT.sample_tokens; HF: the fused head), with the
            # logits it drew from
            with plan_trace() as tr:
                sampled, selp, logits = draw_fn(s, gum.to(cuda))
                torch.cuda.synchronize()
            if kind == "hf":
                assert tr.has("tied_logits_sample"), tr.lines
            ref = ref_fn(s.cpu())
            assert logits.shape == ref.shape == (NUM, n0, K)
            e = rel(logits, ref)
            assert e < 1e-4, f"{kind} step {t}: logits rel err {e}"
            sc = s.cpu()
            want, sel = O.race_sample(logits.cpu(), sc, K, gum)
            assert torch.equal(sampled.cpu(), want), f"{kind} step {t}: draws differ"
            unk = sc == K
            ps = selp.cpu()
            assert torch.isinf(ps[~unk]).all()
            pe = float(((ps[unk].double() - sel[unk]).abs() / sel[unk]).max())
            assert pe < 2e-6, f"{kind} step {t}: p(sampled) rel err {pe}"
            u_g = torch.rand(NUM, n0, generator=g)
            ratio = (t + 1) / T
            k = mask_len(n0, O.gamma_cosine(ratio))
            want = O.remask_step(ps, want, K, t, T, torch.full((NUM,), n0), temp, u_g)
            s = maskgit_remask(selp, k, temp * (1.0 - ratio), sampled, K, u_gumbel=u_g.to(cuda))
            got = s.cpu()
            assert torch.equal(got, want), (
                f"{kind} step {t}: {(got != want).sum().item()} tokens differ from the oracle")
            assert int((got == K).sum(1).max()) == k == int((got == K).sum(1).min())
        return s

    with torch.no_grad():
        K = mg.mask_token_ids["lf"]
        s_l = torch.full((NUM, 24), K, dtype=torch.int64, device=cuda)
        s_l = drive("lf", s_l, mg.T["lf"], mg.choice_temperature_l, 24,
                    lambda s, gum: mg.sample_tokens(mg.transformer_l, None, K, s, gumbel=gum,
                                                    want_logits=True),
                    lambda s: O.transformer_forward(ctx, sd_l, "lf", s, None, null, K,
                                                    pl["heads"], pl["n_layers"]))
        s_lc = s_l.cpu()
        assert int(s_lc.max()) < K and int(s_lc.min()) >= 0  # every LF token decoded
        Kh = mg.mask_token_ids["hf"]
        s_h = torch.full((NUM, 96), Kh, dtype=torch.int64, device=cuda)
        s_h = drive("hf", s_h, mg.T["hf"], mg.choice_temperature_h, 96,
                    lambda s, gum: mg.sample_tokens(mg.transformer_h, None, Kh, s_l, s,
                                                    gumbel=gum, want_logits=True),
                    lambda s: O.transformer_forward(ctx, sd_h, "hf", s_lc, s, null, Kh,
                                                    ph["heads"], ph["n_layers"]))
        s_hc = s_h.cpu()
        assert int(s_hc.max()) < Kh and int(s_hc.min()) >= 0  # every HF token decoded

        # decode to series: the 64-row subset against the oracle decoder (eval BN)
        spec = O.Stage1Spec(256, 6)
        x_l = mg.decode_token_ind_to_timeseries(s_l, "lf")
        x_h = mg.decode_token_ind_to_timeseries(s_h, "hf")
        assert x_l.shape == x_h.shape == (NUM, 6, 256)
        rows = torch.randperm(NUM, generator=g)[:64]
        for band, s_c, x_d, dec, vq, plan, bf in (
                ("lf", s_lc, x_l, mg.decoder_l, mg.vq_model_l, spec.dec_l, O.band_lf),
                ("hf", s_hc, x_h, mg.decoder_h, mg.vq_model_h, spec.dec_h, O.band_hf)):
            E = vq._codebook.embed.detach().cpu()
            H = 3
            W = s_c.shape[1] // H
            zq = E[s_c[rows]].transpose(1, 2).reshape(64, E.shape[1], H, W)
            ref = O.decoder_forward(ctx, _state(dec), "", zq, plan, bf, 6, 256)
            got = x_d[rows.to(cuda)]
            e = rel(got, ref)
            assert e < 1e-4, f"{band} decode rel err {e}"
            assert float((got.cpu() - ref).abs().max()) <= 1e-4 * (1.0 + float(ref.abs().max()))


def test_graphed_sampler_1024_equals_eager(mg, cuda):
    from timevqvae.hip import rng
    from timevqvae.utils.sample_utils import GraphedSampler
    gs = GraphedSampler(mg, NUM, cuda)
    rng.manual_seed(31)
    got = [t.clone() for t in gs.sample()]
    again = [t.clone() for t in gs.sample()]
    rng.manual_seed(31)
    with torch.no_grad():
        rng.advance(cuda)
        s_l, s_h = mg.iterative_decoding(num=NUM, device=cuda)
        x_l = mg.decode_token_ind_to_timeseries(s_l, "lf")
        x_h = mg.decode_token_ind_to_timeseries(s_h, "hf")
    K_l, K_h = mg.mask_token_ids["lf"], mg.mask_token_ids["hf"]
    assert s_l.shape == (NUM, 24) and s_h.shape == (NUM, 96)
    assert int(s_l.max()) < K_l and int(s_l.min()) >= 0
    assert int(s_h.max()) < K_h and int(s_h.min()) >= 0
    for a, b in zip(got, (x_l, x_h, x_l + x_h)):
        assert torch.equal(a, b)
    assert torch.equal(got[2], got[0] + got[1])
    assert all(torch.isfinite(t).all() for t in got)
    assert not torch.equal(again[2], got[2])  # the device seed advances per replay
    # the codes used are spread (a collapsed sampler would repeat one code)
    assert len(torch.unique(s_l)) > 32 and len(torch.unique(s_h)) > 32


def test_unconditional_sample_1024(mg, cuda):
    """utils/sample_utils.unconditional_sample at the sampler's batch: ragged last batch,
    representations, one host transfer; x == x_l + x_h on the host."""
    from timevqvae.utils.sample_utils import unconditional_sample
    (x_l, x_h, x), (q_l, q_h) = unconditional_sample(mg, NUM + 100, cuda, batch_size=NUM,
                                                      return_representations=True)
    assert x_l.device.type == "cpu" and x.shape == (NUM + 100, 6, 256)
    assert q_l.shape == (NUM + 100, 128, 3, 8) and q_h.shape == (NUM + 100, 128, 3, 32)
    assert torch.equal(x, x_l + x_h)
    assert bool(torch.isfinite(x).all())
    # the decoder run on the returned latents reproduces the series (eval BN: rows independent)
    with torch.no_grad():
        again = mg.decoder_l(q_l[:64].to(cuda)).cpu()
    assert rel(again, x_l[:64]) < 1e-5
