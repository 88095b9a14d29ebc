"""FID (evaluation/eval_utils.py:56-81) against the reference's own calculate_fid (G10,
tests/golden/make_golden.py gen_fid): the oracle restatement on CPU, and the HIP float64
moments (mean, sample covariance) + host sqrtm on the GPU.  Tolerances: moments rel 1e-10
(float64, different summation order); FID rel 1e-9 for float64 features, 1e-5 for the
float32 case (the reference averages float32 features in float32, the device in float64)."""
import numpy as np
import pytest

from conftest import golden

CASES = ["a", "b", "c"]


@pytest.mark.parametrize("k", CASES)
def test_oracle_fid_matches_reference(k):
    from oracle import tvq_oracle as O
    g = golden("g10_fid.npz")
    np.testing.assert_allclose(O.fid(g[f"{k}_z1"], g[f"{k}_z2"]), g[f"{k}_fid"], rtol=1e-10)


@pytest.mark.gpu
@pytest.mark.parametrize("k", CASES)
def test_device_fid_matches_reference(k):
    from timevqvae.evaluation import calculate_fid, feature_moments
    g = golden("g10_fid.npz")
    for i in (1, 2):
        mu, sigma = feature_moments(g[f"{k}_z{i}"])
        np.testing.assert_allclose(mu.cpu().numpy(), g[f"{k}_mu{i}"], rtol=1e-6 if k == "c" else 1e-10,
                                   atol=1e-7 if k == "c" else 1e-12)
        np.testing.assert_allclose(sigma.cpu().numpy(), g[f"{k}_sigma{i}"], rtol=1e-10, atol=1e-12)
    fid = calculate_fid(g[f"{k}_z1"], g[f"{k}_z2"])
    np.testing.assert_allclose(fid, g[f"{k}_fid"], rtol=1e-5 if k == "c" else 1e-9)


@pytest.mark.gpu
def test_device_fid_identical_sets_is_zero_and_symmetric():
    from timevqvae.evaluation import calculate_fid
    rng = np.random.default_rng(0)
    z = rng.standard_normal((300, 40))
    w = rng.standard_normal((250, 40)) * 1.3 + 0.2
    assert abs(calculate_fid(z, z)) < 1e-8
    np.testing.assert_allclose(calculate_fid(z, w), calculate_fid(w, z), rtol=1e-9)


@pytest.mark.gpu
def test_device_moments_large_feature_dim():
    """ROCKET-sized features (D = 2 x 1000 kernels) against numpy."""
    import torch
    from timevqvae.evaluation import feature_moments
    rng = np.random.default_rng(1)
    z = rng.standard_normal((1100, 2000))
    mu, sigma = feature_moments(torch.from_numpy(z).cuda())
    np.testing.assert_allclose(mu.cpu().numpy(), z.mean(0), rtol=1e-10, atol=1e-13)
    np.testing.assert_allclose(sigma.cpu().numpy(), np.cov(z, rowvar=False), rtol=1e-9, atol=1e-12)
