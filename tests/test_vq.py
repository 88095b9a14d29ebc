"""VQ codebook: oracle pinned to the reference goldens (CPU) and the HIP path vs oracle (GPU).

Index parity rule (SURVEY §7 "Index-exact argmin"): every code index must equal the
oracle's unless the row's fp64 top-2 distance gap is inside the fp32 rounding bound
of the distance expansion, GAP_TOL = 1e-5 * (|x|^2 + max|e|^2)  (documented bound).
"""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import vq_ref


def gap_tol(x, E):
    return 1e-5 * ((x.astype(np.float64) ** 2).sum(1) + (E.astype(np.float64) ** 2).sum(1).max())


def assert_index_parity(got, want, gap, tol, what):
    bad = np.nonzero(got != want)[0]
    unexplained = [int(i) for i in bad if gap[i] > tol[i]]
    assert not unexplained, (
        f"{what}: {len(unexplained)} index mismatches outside the fp32 bound, e.g. rows "
        f"{unexplained[:5]} gaps {[float(gap[i]) for i in unexplained[:5]]}")


# ----------------------------------------------------------------------------- CPU
@pytest.mark.parametrize("variant", ["random", "near"])
def test_oracle_vq_matches_reference_golden(variant):
    g = golden(f"g1_vq_{variant}.npz")
    x = g["x"].reshape(-1, g["x"].shape[-1])
    idx, _, gap = vq_ref.assign(x, g["embed"])
    assert (idx == g["ind"].reshape(-1)).all()
    assert (idx == g["eval_ind"].reshape(-1)).all()
    cs, ea, E, counts, perp = vq_ref.ema(x, idx, g["cluster_size"], g["embed_avg"])
    np.testing.assert_allclose(cs, g["post_cluster_size"], rtol=1e-6, atol=1e-5)
    np.testing.assert_allclose(ea, g["post_embed_avg"], rtol=1e-5, atol=1e-5)
    rown = np.linalg.norm(g["post_embed"], axis=1, keepdims=True)
    assert (np.abs(E - g["post_embed"]) / rown).max() < 1e-5
    assert abs(perp - float(g["perplexity"])) / float(g["perplexity"]) < 1e-4


def test_oracle_vq_kat():
    """The reference's own __main__ known answer (vq.py:410-424): ind[0][0] == 87."""
    k = golden("g0_vq_kat.npz")
    torch.manual_seed(0)
    x = torch.rand((1024, 32, 128))
    E = torch.randn(512, 128)  # EuclideanCodebook init draw (vq.py:145-146)
    idx, _, _ = vq_ref.assign(x.reshape(-1, 128).numpy(), E.numpy())
    assert (idx.reshape(1024, 32)[0] == k["kat_ind0"]).all()
    assert len(np.unique(idx)) == int(k["kat_n_unique"])


# ----------------------------------------------------------------------------- GPU
def _vq_module(K, D, cuda, embed=None, embed_avg=None, cluster_size=None):
    from timevqvae.models import VectorQuantize
    vq = VectorQuantize(D, K).to(cuda)
    if embed is not None:
        vq._codebook.embed.copy_(torch.from_numpy(embed))
        vq._codebook.embed_avg.copy_(torch.from_numpy(embed_avg))
        vq._codebook.cluster_size.copy_(torch.from_numpy(cluster_size))
    return vq


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["random", "near"])
def test_hip_vq_matches_reference_golden(variant, cuda):
    g = golden(f"g1_vq_{variant}.npz")
    K, D = g["embed"].shape
    vq = _vq_module(K, D, cuda, g["embed"], g["embed_avg"], g["cluster_size"])
    x = torch.from_numpy(g["x"]).to(cuda)
    xf = x.reshape(-1, D).cpu().numpy()
    tol = gap_tol(xf, g["embed"])
    vq.eval()
    q, ind, _, perp = vq(x)
    assert_index_parity(ind.cpu().numpy().reshape(-1), g["eval_ind"].reshape(-1), g["gap64"], tol,
                        "eval")
    np.testing.assert_array_equal(q.cpu().numpy(), g["embed"][ind.cpu().numpy()])
    assert abs(float(perp) - float(g["eval_perplexity"])) <= 1e-4 * float(g["eval_perplexity"])
    vq.train()
    xg = x.clone().requires_grad_(True)
    q, ind, loss, perp = vq(xg)
    (q.square().sum() * 0.5 + loss["loss"].sum()).backward()
    torch.cuda.synchronize()
    ind_np = ind.cpu().numpy().reshape(-1)
    assert_index_parity(ind_np, g["ind"].reshape(-1), g["gap64"], tol, "train")
    assert (ind_np == g["ind"].reshape(-1)).all(), "golden rows have no near-ties: must be exact"
    np.testing.assert_allclose(float(loss["commit_loss"]), float(g["commit"]), rtol=1e-4)
    np.testing.assert_allclose(float(perp), float(g["perplexity"]), rtol=1e-4)
    cb = vq._codebook
    np.testing.assert_allclose(cb.cluster_size.cpu().numpy(), g["post_cluster_size"], rtol=1e-5,
                               atol=1e-5)
    np.testing.assert_allclose(cb.embed_avg.cpu().numpy(), g["post_embed_avg"], rtol=1e-4,
                               atol=1e-5)
    rown = np.linalg.norm(g["post_embed"], axis=1, keepdims=True)
    assert (np.abs(cb.embed.cpu().numpy() - g["post_embed"]) / rown).max() < 1e-4
    np.testing.assert_allclose(xg.grad.cpu().numpy(), g["x_grad"], rtol=1e-4, atol=1e-6)


@pytest.mark.gpu
def test_hip_vq_kat(cuda):
    """vq.py:410-424 known answer, through the product module on the GPU."""
    k = golden("g0_vq_kat.npz")
    from timevqvae.models import VectorQuantize
    torch.manual_seed(0)
    x = torch.rand((1024, 32, 128))
    vq = VectorQuantize(dim=128, codebook_size=512)
    vq = vq.to(cuda)
    q, ind, loss, perp = vq(x.to(cuda))
    ind = ind.cpu().numpy()
    assert (ind[0] == k["kat_ind0"]).all()
    assert len(np.unique(ind)) == int(k["kat_n_unique"])
    np.testing.assert_allclose(float(loss["commit_loss"]), float(k["kat_commit"]), rtol=1e-4)
    np.testing.assert_allclose(float(perp), float(k["kat_perplexity"]), rtol=1e-4)
    np.testing.assert_allclose(float(vq._codebook.cluster_size.sum()), float(k["kat_cs_sum"]),
                               rtol=1e-5)
    np.testing.assert_allclose(vq._codebook.embed[0, :4].cpu().numpy(), k["kat_embed0"], rtol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("M,K,D,layout", [
    (24576, 512, 128, "nchw"),   # config B HF tokens (256 x 96), strided NCHW view
    (6144, 512, 128, "rows"),    # config B LF tokens, row-major
    (1000, 37, 64, "rows"),      # ragged: M, K not multiples of the tiles
    (77, 16, 32, "nchw"),
])
def test_hip_vq_vs_c_oracle_full_size(M, K, D, layout, cuda):
    rng = np.random.default_rng(M + K)
    if layout == "nchw":
        HW = 96 if M % 96 == 0 else 7
        Bb = M // HW
        M = Bb * HW
        z = torch.from_numpy(rng.standard_normal((Bb, D, 1, HW)).astype(np.float32)).to(cuda)
        x = z.flatten(2).transpose(1, 2)  # (B, HW, D) strided view, as quantize() makes it
    else:
        x = torch.from_numpy(rng.standard_normal((M, D)).astype(np.float32)).to(cuda).reshape(1, M, D)
    E = rng.standard_normal((K, D)).astype(np.float32)
    ea = E + 0.01 * rng.standard_normal((K, D)).astype(np.float32)
    cs = rng.uniform(0, 2, K).astype(np.float32)
    vq = _vq_module(K, D, cuda, E, ea, cs)
    xh = x.reshape(-1, D).cpu().numpy()
    want, _, gap = vq_ref.assign(xh, E)
    vq.train()
    q, ind, loss, perp = vq(x)
    torch.cuda.synchronize()
    got = ind.cpu().numpy().reshape(-1)
    assert_index_parity(got, want, gap, gap_tol(xh, E), f"M={M} K={K} D={D}")
    # and against the reference's own fp32 expression (vq.py:210-222) on the same x
    from test_fullsize_parity import ref_expr_flips
    assert ref_expr_flips(x, torch.from_numpy(E), ind, f"vq M={M} K={K} D={D}") == 0
    cs2, ea2, E2, counts, p = vq_ref.ema(xh, got, cs, ea)
    np.testing.assert_allclose(vq._codebook.cluster_size.cpu().numpy(), cs2, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(vq._codebook.embed_avg.cpu().numpy(), ea2, rtol=1e-4, atol=1e-4)
    rown = np.linalg.norm(E2, axis=1, keepdims=True)
    assert (np.abs(vq._codebook.embed.cpu().numpy() - E2) / rown).max() < 1e-4
    np.testing.assert_allclose(float(perp), p, rtol=1e-4)
    qs = q.detach().reshape(-1, D).cpu().numpy()
    np.testing.assert_allclose(qs, E[got], rtol=1e-6, atol=1e-6)  # straight-through value ~= q
    commit = ((xh.astype(np.float64) - E[got]) ** 2).mean()
    np.testing.assert_allclose(float(loss["commit_loss"]), commit, rtol=1e-4)


@pytest.mark.gpu
def test_hip_vq_layout_independent(cuda):
    """Strided NCHW view and a contiguous copy give identical indices and outputs."""
    rng = np.random.default_rng(3)
    z = torch.from_numpy(rng.standard_normal((64, 128, 3, 32)).astype(np.float32)).to(cuda)
    E = rng.standard_normal((512, 128)).astype(np.float32)
    a = _vq_module(512, 128, cuda, E, E, np.zeros(512, np.float32)).eval()
    xv = z.flatten(2).transpose(1, 2)
    q1, i1, _, _ = a(xv)
    q2, i2, _, _ = a(xv.contiguous())
    assert torch.equal(i1, i2)
    assert torch.equal(q1, q2)


# ----------------------------------------------------------------------------- stochastic VQ
def _svq_oracle(g6, key, train):
    """The oracle's VectorQuantize pass with svq_temp under the golden's seed."""
    from oracle import tvq_oracle as O
    E = torch.from_numpy(g6["embed"])
    sd = {"_codebook.embed": E, "_codebook.cluster_size": torch.zeros(E.shape[0]),
          "_codebook.embed_avg": E.clone()}
    ctx = O.Ctx(training=train)
    torch.manual_seed(int(g6[f"{key}_seed"]))
    q, ind, _, perp = O.vq_forward(ctx, sd, "", torch.from_numpy(g6["x"]),
                                   svq_temp=float(g6[f"{key}_temp"]))
    return ind, perp, ctx.updates


@pytest.mark.parametrize("j", [0, 1])
@pytest.mark.parametrize("mode", ["eval", "train"])
def test_oracle_svq_matches_reference_golden(j, mode):
    """G6: the reference's Categorical draws (vq.py:51-56,216-222) reproduced by the oracle
    restatement under the same torch seed, including the EMA that follows them."""
    g6 = golden("g6_svq.npz")
    key = f"t{j}_{mode}"
    ind, perp, upd = _svq_oracle(g6, key, mode == "train")
    assert (ind.numpy() == g6[f"{key}_ind"]).all()
    assert abs(float(perp) - float(g6[f"{key}_perplexity"])) < 1e-4 * float(perp)
    if mode == "train":
        np.testing.assert_allclose(upd["_codebook.cluster_size"].numpy(),
                                   g6[f"{key}_post_cluster_size"], rtol=1e-6, atol=1e-6)
        np.testing.assert_allclose(upd["_codebook.embed"].numpy(), g6[f"{key}_post_embed"],
                                   rtol=1e-5, atol=1e-5)


def test_oracle_svq_gumbel_form_is_the_same_distribution():
    """Gumbel-max (the HIP path's draw) and Categorical (the reference's) sample the same
    softmax(dist/temp): empirical frequencies over 20k draws of one row agree within 5 sigma."""
    from oracle import tvq_oracle as O
    g = torch.Generator().manual_seed(7)
    E = torch.randn(16, 8, generator=g)
    x = torch.randn(1, 8, generator=g)
    temp = 3.0
    dist = O.vq_dist(x, E)
    p = torch.softmax(dist.double() / temp, -1)[0]
    n = 20000
    u = torch.rand(n, 16, generator=g, dtype=torch.float64).clamp_min(1e-300)
    gum = (-torch.log(-torch.log(u))).float()
    idx, _ = O.vq_sample_gumbel(dist.expand(n, -1), temp, gum)
    freq = torch.bincount(idx, minlength=16).double() / n
    sigma = torch.sqrt(p * (1 - p) / n)
    assert ((freq - p).abs() <= 5 * sigma + 1e-4).all()


@pytest.mark.gpu
@pytest.mark.parametrize("temp", [0.5, 4.0])
def test_hip_svq_injected_noise_vs_oracle(temp, cuda):
    """Device Gumbel-max with injected noise == oracle argmax(dist/temp + g), except where
    the fp64 top-2 gap of the perturbed logits is inside the fp32 distance bound / temp."""
    from oracle import tvq_oracle as O
    from timevqvae.hip.vq import vq_codebook_pass
    g6 = golden("g6_svq.npz")
    x = torch.from_numpy(g6["x"])
    E = torch.from_numpy(g6["embed"])
    M, K = x.shape[1], E.shape[0]
    gen = torch.Generator().manual_seed(11)
    gum = -torch.log(-torch.log(torch.rand(M, K, generator=gen).clamp(1e-7, 1 - 1e-7)))
    want, gap = O.vq_sample_gumbel(O.vq_dist(x[0], E), temp, gum)
    cs = torch.zeros(K, device=cuda)
    _, idx, _, _, counts = vq_codebook_pass(
        x.to(cuda), E.to(cuda), cs, E.clone().to(cuda), straight_through=False, ema=False,
        decay=0.8, eps=1e-5, svq_temp=temp, gumbel=gum.to(cuda))
    got = idx.reshape(-1).cpu().numpy()
    tol = gap_tol(x[0].numpy(), E.numpy()) / temp + 1e-6
    assert_index_parity(got, want.numpy(), gap.numpy(), tol, f"svq temp={temp}")
    assert int(counts.sum()) == M


@pytest.mark.gpu
def test_hip_svq_device_rng_distribution(cuda):
    """Device-seeded draws follow softmax(dist/temp) (the reference's Categorical): one row
    replicated 32768 times, per-code frequencies within 5 sigma of the oracle's fp64 softmax;
    temp -> 0 is the deterministic argmax; successive calls draw different samples."""
    from oracle import tvq_oracle as O
    from timevqvae.models import VectorQuantize
    g = torch.Generator().manual_seed(5)
    D, K, n = 32, 64, 32768
    E = torch.randn(K, D, generator=g) * 0.3
    row = torch.randn(1, D, generator=g) * 0.3
    temp = 2.0
    p = torch.softmax(O.vq_dist(row, E).double() / temp, -1)[0]
    vq = VectorQuantize(D, K).to(cuda).eval()
    vq._codebook.embed.copy_(E)
    x = row.expand(n, D).reshape(1, n, D).contiguous().to(cuda)
    _, ind, _, _ = vq(x, svq_temp=temp)
    freq = torch.bincount(ind.reshape(-1).cpu(), minlength=K).double() / n
    sigma = torch.sqrt(p * (1 - p) / n)
    assert ((freq - p).abs() <= 5 * sigma + 2e-4).all(), (freq - p).abs().max()
    _, ind2, _, _ = vq(x, svq_temp=temp)
    assert (ind2 != ind).any()
    _, ind0, _, _ = vq(x, svq_temp=None)
    assert (ind0 == int(p.argmax())).all()


@pytest.mark.gpu
def test_hip_svq_training_ema_uses_sampled_indices(cuda):
    """Training with svq_temp: the EMA statistics follow the sampled indices (vq.py:227-245),
    checked against the C oracle's EMA on the device's own draws."""
    from timevqvae.models import VectorQuantize
    g6 = golden("g6_svq.npz")
    x = g6["x"]
    E = g6["embed"]
    K, D = E.shape
    vq = _vq_module(K, D, cuda, embed=E, embed_avg=E.copy(), cluster_size=np.zeros(K, np.float32))
    vq.train()
    xt = torch.from_numpy(x).to(cuda).requires_grad_(True)
    q, ind, loss, perp = vq(xt, svq_temp=4.0)
    torch.cuda.synchronize()
    cs, ea, Enew, counts, p = vq_ref.ema(x.reshape(-1, D), ind.reshape(-1).cpu().numpy(),
                                          np.zeros(K, np.float32), E)
    np.testing.assert_allclose(vq._codebook.cluster_size.cpu().numpy(), cs, rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(vq._codebook.embed.cpu().numpy(), Enew, rtol=1e-5, atol=1e-5)
    assert abs(float(perp) - p) < 1e-4 * p
    # the straight-through output is the (pre-update) codeword of the sampled index
    np.testing.assert_allclose(q.detach().cpu().numpy()[0], E[ind.reshape(-1).cpu().numpy()],
                               rtol=0, atol=2e-6)


@pytest.mark.gpu
def test_hip_vq_nan_rows_match_torch_argmax(cuda):
    """NaN distances: torch.argmax (vq.py:216-222) treats NaN as the maximum and returns the
    first NaN index. A NaN token row therefore maps to code 0, and a NaN codebook row k
    to code k for every token (the first NaN of each row)."""
    from timevqvae.models import VectorQuantize
    torch.manual_seed(3)
    K, D = 64, 128
    x = torch.randn(2, 16, D)
    x[0, 3] = float("nan")
    x[1, 7, 5] = float("nan")
    E = torch.randn(K, D)
    E[9] = float("nan")
    E[40, 0] = float("nan")

    def ref(xx, EE):
        flat = xx.reshape(-1, D)
        dist = -(flat.pow(2).sum(1, keepdim=True) - 2 * flat @ EE.t() + EE.pow(2).sum(1)[None])
        return dist.argmax(-1).reshape(xx.shape[:-1])

    for EE in (torch.randn(K, D), E):
        vq = VectorQuantize(D, K).to(cuda).eval()
        vq._codebook.embed.copy_(EE)
        _, ind, _, _ = vq(x.to(cuda))
        want = ref(x, EE)
        assert (ind.cpu() == want).all(), (ind.cpu()[want != ind.cpu()], want[want != ind.cpu()])
