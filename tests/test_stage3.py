"""Stage3 / FidelityEnhancer training (trainers/stage3.py:193-231,
models/fidelity_enhancer.py:96-498) against G11, made by the reference's own files
(tests/golden/make_golden.py gen_fe_train, dropout 0):
  a / b  FidelityEnhancer train forward + L1 + backward at input_length 256 / 301;
  s3     the reference Stage3._fidelity_enhancer_loss_fn (MaskGIT decode of LF / HF token
         indices over the G3-small stage1, FE, L1) and every FE gradient.
fp32 tolerances: outputs and losses |d| <= 1e-4 (1 + |ref|); gradients per tensor
|d|max <= 2e-4 max|ref| + 1e-6 (a deep net of GroupNorms: summation order differs).
Dropout (p = 0.5, the config's) is checked for mask consistency on the op level."""
import numpy as np
import pytest
import torch

from conftest import golden
from param_init import fill_state_dict

CFG = {"dim": 8, "dim_mults": [1, 2, 4, 8], "resnet_block_groups": 4, "dropout": 0.0,
       "tau_search_rng": [0.1, 0.5, 1, 2, 4], "tau_search_subset_size": 1.0,
       "percept_loss_weight": 0.0}


def _fe(C, Lin, seed, dropout=0.0):
    from timevqvae.models import FidelityEnhancer
    fe = FidelityEnhancer(Lin, C, {"fidelity_enhancer": dict(CFG, dropout=dropout)})
    vals = fill_state_dict(fe.state_dict(), seed)
    fe.load_state_dict({k: torch.from_numpy(v) for k, v in vals.items()})
    return fe


def _close(got, want, what):
    err = np.abs(got - want) - 1e-4 * (1 + np.abs(want))
    assert float(err.max()) <= 0, (what, float(np.abs(got - want).max()))


def _grads_close(named, g, prefix):
    n = 0
    for k, p in named:
        key = f"{prefix}grad/{k}"
        if key not in g:
            assert p.grad is None or float(p.grad.abs().max()) == 0.0, k
            continue
        ref = g[key]
        got = p.grad.detach().cpu().numpy()
        tol = 2e-4 * float(np.abs(ref).max()) + 1e-6
        assert float(np.abs(got - ref).max()) <= tol, (k, float(np.abs(got - ref).max()), tol)
        n += 1
    assert n == len([k for k in g if k.startswith(prefix + "grad/")])


def test_g11_gradient_keys_are_the_fe_parameters():
    g = golden("g11_fe_train.npz")
    fe = _fe(6, 256, 21)
    names = {k for k, _ in fe.named_parameters()}
    for tag in ("a", "s3"):
        keys = {k[len(tag) + 6:] for k in g if k.startswith(f"{tag}_grad/")}
        assert keys and keys <= names


@pytest.mark.gpu
@pytest.mark.parametrize("tag", ["a", "b"])
def test_fe_train_step_vs_reference(tag, cuda):
    from timevqvae.hip.loss import l1_loss
    g = golden("g11_fe_train.npz")
    B, C, Lx, Lin, seed = (int(v) for v in g[f"{tag}_meta"])
    fe = _fe(C, Lin, seed).to(cuda).train()
    xp = torch.from_numpy(g[f"{tag}_xprime"]).to(cuda)
    x = torch.from_numpy(g[f"{tag}_x"]).to(cuda)
    xhat = fe(xp)
    loss = l1_loss(xhat, x)
    loss.backward()
    _close(xhat.detach().cpu().numpy(), g[f"{tag}_xhat"], "xhat")
    _close(np.array(float(loss)), g[f"{tag}_loss"], "loss")
    _grads_close(fe.named_parameters(), g, f"{tag}_")


def _stage3(cuda, dropout=0.0, feature_extractor_type="supervised_fcn"):
    from test_stage2_golden import _maskgit
    from timevqvae.trainers import Stage3
    mg = _maskgit(cuda)

    class _S2(torch.nn.Module):
        def __init__(self, m):
            super().__init__()
            self.maskgit = m
    cfg = {"VQ-VAE": {"n_fft": 4}, "fidelity_enhancer": dict(CFG, dropout=dropout),
           "exp_params": {"lr": 1e-3, "linear_warmup_rate": 0.1},
           "trainer_params": {"max_steps": {"stage3": 100}}}
    st = Stage3(None, None, None, 128, 6, 5, config=cfg, stage2=_S2(mg), device=cuda,
                feature_extractor_type=feature_extractor_type)
    vals = fill_state_dict(st.fidelity_enhancer.state_dict(), 23)
    st.fidelity_enhancer.load_state_dict({k: torch.from_numpy(v) for k, v in vals.items()})
    return st.to(cuda)


@pytest.mark.gpu
def test_stage3_loss_fn_vs_reference(cuda):
    g = golden("g11_fe_train.npz")
    st = _stage3(cuda)
    st.eval()
    st.fidelity_enhancer.train()
    x = torch.from_numpy(g["s3_x"]).to(cuda)
    s_l, s_h = (torch.from_numpy(g[k]).to(cuda) for k in ("s3_s_l", "s3_s_h"))
    loss, (xprime, xhat) = st._fidelity_enhancer_loss_fn(x, s_l, s_h)
    loss.backward()
    _close(xprime.cpu().numpy(), g["s3_xprime"], "xprime (MaskGIT decode)")
    _close(xhat.detach().cpu().numpy(), g["s3_xhat"], "xhat")
    _close(np.array(float(loss)), g["s3_loss"], "loss")
    _grads_close(st.fidelity_enhancer.named_parameters(), g, "s3_")
    assert all(p.grad is None for p in st.maskgit.parameters())


@pytest.mark.gpu
def test_stage3_training_steps_update_only_the_fe(cuda):
    """Three optimizer steps at the config's dropout (0.5) and tau 0.5: finite losses, the
    FE moves, the frozen MaskGIT does not."""
    st = _stage3(cuda, dropout=0.5)
    st.fidelity_enhancer.tau = torch.tensor(0.5, device=cuda)
    opt = st.configure_optimizers()["optimizer"]
    g = torch.Generator().manual_seed(5)
    x = torch.cumsum(0.1 * torch.randn(8, 6, 128, generator=g), -1).to(cuda)
    mg0 = [p.detach().clone() for p in st.maskgit.parameters()]
    fe0 = [p.detach().clone() for p in st.fidelity_enhancer.parameters()]
    for i in range(3):
        opt.zero_grad()
        out = st.training_step((x, None), i)
        assert torch.isfinite(out["loss"]).item()
        out["loss"].backward()
        opt.step()
    assert all(torch.equal(a, p) for a, p in zip(mg0, st.maskgit.parameters()))
    assert any(not torch.equal(a, p) for a, p in zip(fe0, st.fidelity_enhancer.parameters()))


@pytest.mark.gpu
def test_gn_snake_dropout_mask_and_gradient(cuda):
    """GroupNorm+Snake+Dropout(0.5) training op: kept outputs are the p=0 output / (1-p),
    dropped ones 0; its gradient equals torch autograd of the same masked expression."""
    from timevqvae.hip import fe_train, rng
    torch.manual_seed(0)
    B, C, L, G = 3, 8, 40, 4
    x = torch.randn(B, C, L, device=cuda, requires_grad=True)
    gam = (1 + 0.1 * torch.randn(C, device=cuda)).requires_grad_()
    bet = (0.1 * torch.randn(C, device=cuda)).requires_grad_()
    a = (0.5 + 0.2 * torch.rand(1, C, 1, device=cuda)).requires_grad_()
    site = rng.new_site()
    y0 = fe_train.group_norm_snake(x, G, gam, bet, a, drop_p=0.0)
    rng._calls[0] = 0
    y = fe_train.group_norm_snake(x, G, gam, bet, a, drop_p=0.5, site=site)
    keep = y != 0
    assert 0.3 < keep.float().mean().item() < 0.7
    torch.testing.assert_close(y[keep], 2 * y0[keep], rtol=1e-6, atol=1e-6)
    gy = torch.randn_like(y)
    dx, dg, db, da = torch.autograd.grad(y, (x, gam, bet, a), gy)
    # torch reference of the same expression with the same mask
    xr, gr, br, ar = (t.detach().clone().requires_grad_() for t in (x, gam, bet, a))
    u = torch.nn.functional.group_norm(xr, G, gr, br, 1e-5)
    s = u + torch.sin(ar * u) ** 2 / ar
    yr = s * keep.float() * 2
    want = torch.autograd.grad(yr, (xr, gr, br, ar), gy)
    for got, w in zip((dx, dg, db, da), want):
        torch.testing.assert_close(got, w, rtol=1e-4, atol=1e-4)


@pytest.mark.gpu
def test_stage3_search_optimal_tau_smoke(cuda):
    g = torch.Generator().manual_seed(6)
    X = torch.cumsum(0.1 * torch.randn(48, 6, 128, generator=g), -1).numpy()
    # the reference's default extractor is the pretrained FCN: no silent ROCKET substitute
    with pytest.raises(NotImplementedError):
        _stage3(cuda).search_optimal_tau(X, cuda, n_samples=16, batch_size=16)
    st = _stage3(cuda, feature_extractor_type="rocket")
    tau = st.search_optimal_tau(X, cuda, n_samples=48, batch_size=16)
    assert tau in CFG["tau_search_rng"]
    assert all(np.isfinite(v) for v in st.tau_fids.values())
    assert abs(float(st.fidelity_enhancer.tau) - float(tau)) < 1e-6
