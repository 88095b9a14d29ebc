"""ROCKET features: evaluation/rocket_functions.py on the GPU.

Pinning: G7 was produced by the reference's own rocket_functions.py (numba stubbed to the
interpreter, float64) — tests/golden/make_golden.py gen_rocket.  The C oracle reproduces
it bit for bit; the HIP transform (float64, unfused, reference order) must equal both
bit for bit, at the golden sizes and at full size on sampled rows.
"""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import rocket_ref

NAMES = ("weights", "lengths", "biases", "dilations", "paddings")


def _kernels(g, tag):
    return tuple(g[f"{tag}_{n}"] for n in NAMES)


@pytest.mark.parametrize("tag", ["a", "b"])
def test_oracle_rocket_matches_reference_golden(tag):
    g = golden("g7_rocket.npz")
    f = rocket_ref.apply_kernels(g[f"{tag}_X"], _kernels(g, tag))
    assert np.array_equal(f, g[f"{tag}_features"])


def test_generate_kernels_matches_reference_draws():
    """Same numpy draws in the reference's order (rocket_functions.py:21-57)."""
    from timevqvae.evaluation import generate_kernels
    g = golden("g7_rocket.npz")
    np.random.seed(7)
    k = generate_kernels(128, 64)
    for a, n in zip(k, NAMES):
        assert np.array_equal(a, g[f"a_{n}"]), n


def test_oracle_threads_agree():
    from timevqvae.evaluation import generate_kernels
    np.random.seed(3)
    k = generate_kernels(200, 30)
    X = np.random.randn(9, 200)
    assert np.array_equal(rocket_ref.apply_kernels(X, k, 1), rocket_ref.apply_kernels(X, k, 4))


@pytest.mark.gpu
@pytest.mark.parametrize("tag", ["a", "b"])
def test_hip_rocket_matches_reference_golden(tag, cuda):
    from timevqvae.evaluation import apply_kernels
    g = golden("g7_rocket.npz")
    f = apply_kernels(g[f"{tag}_X"], _kernels(g, tag), device=cuda)
    want = g[f"{tag}_features"]
    bad = np.argwhere(f != want)
    assert len(bad) == 0, (len(bad), bad[:4].tolist(), f[tuple(bad[0])], want[tuple(bad[0])])


@pytest.mark.gpu
def test_hip_rocket_full_size_sampled_rows(cuda):
    """BASELINE-scale evaluation batch: 1024 series x 10000 kernels at L=256 on the GPU;
    every feature of 8 sampled rows equal to the C oracle's."""
    from timevqvae.evaluation import DeviceKernels, apply_kernels_device, generate_kernels
    np.random.seed(11)
    k = generate_kernels(256, 10000)
    X = np.cumsum(np.random.randn(1024, 256), axis=1)
    dk = DeviceKernels(k, cuda)
    f = apply_kernels_device(torch.from_numpy(X).to(cuda), dk).cpu().numpy()
    rows = np.random.default_rng(0).choice(1024, 8, replace=False)
    want = rocket_ref.apply_kernels(X[rows], k, threads=8)
    assert np.array_equal(f[rows], want)
    assert np.isfinite(f).all()


@pytest.mark.gpu
def test_hip_rocket_strided_input_and_single_kernel(cuda):
    from timevqvae.evaluation import DeviceKernels, apply_kernel, apply_kernels_device
    from timevqvae.evaluation import generate_kernels
    np.random.seed(5)
    k = generate_kernels(64, 12)
    X = np.random.randn(4, 80)
    Xt = torch.from_numpy(X).to(cuda)[:, 8:72]  # row stride 80, length 64
    f = apply_kernels_device(Xt, DeviceKernels(k, cuda)).cpu().numpy()
    assert np.array_equal(f, rocket_ref.apply_kernels(X[:, 8:72], k))
    w, lengths, biases, dil, pad = k
    ppv, mx = apply_kernel(X[1, 8:72], w[:lengths[0]], lengths[0], biases[0], dil[0], pad[0])
    assert (ppv, mx) == (f[1, 0], f[1, 1])


def test_rocket_rejects_kernels_outside_contract():
    from timevqvae.evaluation import DeviceKernels
    k = (np.zeros(17), np.array([17], np.int32), np.zeros(1), np.ones(1, np.int32),
         np.zeros(1, np.int32))
    with pytest.raises(ValueError):
        DeviceKernels(k, "cpu")
