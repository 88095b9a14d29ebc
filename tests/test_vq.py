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
