"""FidelityEnhancer / Unet1D eval forward (models/fidelity_enhancer.py).

Pinning: G8 was produced by the reference's own fidelity_enhancer.py (loaded by file path,
configs/config.yaml:69-77 hyper-parameters, param_init's per-key weights) —
tests/golden/make_golden.py gen_fe.  The oracle restatement (oracle/tvq_oracle.py
fe_forward) must reproduce G8; the HIP forward must match G8 and, at the sampler's batch,
the oracle.  fp32 tolerance: |got - want| <= 1e-4 * (1 + |want|) elementwise (summation
order of convs / norms differs from torch CPU).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import golden
from oracle import tvq_oracle as O
from param_init import fill_state_dict

CFG = {"fidelity_enhancer": {"dim": 8, "dim_mults": [1, 2, 4, 8], "resnet_block_groups": 4,
                             "dropout": 0.5, "tau_search_rng": [0.1, 0.5]}}
ATOL, RTOL = 1e-4, 1e-4


def _model(C, Lin, seed):
    from timevqvae.models import FidelityEnhancer
    fe = FidelityEnhancer(Lin, C, CFG)
    vals = fill_state_dict(fe.state_dict(), seed)
    fe.load_state_dict({k: torch.from_numpy(v) for k, v in vals.items()})
    return fe.eval()


def _close(got, want):
    err = np.abs(got - want) - (ATOL + RTOL * np.abs(want))
    return float(err.max()) <= 0, float(np.abs(got - want).max())


def test_state_dict_keys_match_reference():
    g = golden("g8_fe.npz")
    fe = _model(6, 256, 11)
    assert sorted(fe.state_dict().keys()) == list(g["a_keys"])


@pytest.mark.parametrize("tag", ["a", "b"])
def test_oracle_fe_matches_reference_golden(tag):
    g = golden("g8_fe.npz")
    B, C, Lx, Lin, seed = (int(v) for v in g[f"{tag}_meta"])
    sd = {k: v.detach() for k, v in _model(C, Lin, seed).state_dict().items()}
    y = O.fe_forward(sd, torch.from_numpy(g[f"{tag}_x"]), Lin).numpy()
    ok, err = _close(y, g[f"{tag}_y"])
    assert ok, err


@pytest.mark.gpu
@pytest.mark.parametrize("tag", ["a", "b"])
def test_hip_fe_matches_reference_golden(tag, cuda):
    g = golden("g8_fe.npz")
    B, C, Lx, Lin, seed = (int(v) for v in g[f"{tag}_meta"])
    fe = _model(C, Lin, seed).to(cuda)
    y = fe(torch.from_numpy(g[f"{tag}_x"]).to(cuda)).cpu().numpy()
    assert y.shape == g[f"{tag}_y"].shape
    ok, err = _close(y, g[f"{tag}_y"])
    assert ok, err


@pytest.mark.gpu
def test_hip_fe_sampler_batch_vs_oracle(cuda):
    """The sampler's batch (1024 trajectories, generation/sampler.py:156-169): 64 rows
    checked against the oracle, the rest for batch independence (same row twice)."""
    torch.manual_seed(0)
    fe = _model(6, 256, 5).to(cuda)
    x = torch.cumsum(0.1 * torch.randn(1024, 6, 256), -1)
    x[1023] = x[5]
    y = fe(x.to(cuda)).cpu()
    sd = {k: v.detach().cpu() for k, v in fe.state_dict().items()}
    want = O.fe_forward(sd, x[:64], 256)
    ok, err = _close(y[:64].numpy(), want.numpy())
    assert ok, err
    assert torch.equal(y[1023], y[5])
    assert torch.isfinite(y).all()
    # the cached standardised weights follow in-place parameter updates
    w = fe.unet.downs[0][0].block1.proj.weight
    with torch.no_grad():
        w.mul_(1.5).add_(0.01)
    sd = {k: v.detach().cpu() for k, v in fe.state_dict().items()}
    ok, err = _close(fe(x[:8].to(cuda)).cpu().numpy(), O.fe_forward(sd, x[:8], 256).numpy())
    assert ok, err


@pytest.mark.gpu
@pytest.mark.parametrize("K,S,P,up2,rep", [(7, 1, 3, 0, 0), (4, 2, 1, 0, 0), (3, 1, 1, 1, 0), (9, 3, 4, 0, 0),
                                          (3, 1, 1, 0, 1), (1, 1, 0, 0, 0)])
def test_hip_conv1d_geometries(K, S, P, up2, rep, cuda):
    from timevqvae.hip import fe as ops
    torch.manual_seed(K * 10 + S)
    for Ci, Co, L in [(6, 8, 256), (96, 32, 37), (8, 67, 130)]:
        x, w, b = torch.randn(3, Ci, L), torch.randn(Co, Ci, K), torch.randn(Co)
        xi = F.interpolate(x, scale_factor=2, mode="nearest") if up2 else x
        want = F.conv1d(F.pad(xi, (P, P), mode="replicate"), w, b, S) if rep \
            else F.conv1d(xi, w, b, S, P)
        got = ops.conv1d(x.to(cuda), w.to(cuda), b.to(cuda), S, P, bool(up2), bool(rep)).cpu()
        assert got.shape == want.shape
        assert torch.allclose(got, want, atol=1e-4, rtol=1e-4), (Ci, Co, L)


@pytest.mark.gpu
def test_hip_fe_norms_and_attention(cuda):
    from timevqvae.hip import fe as ops
    torch.manual_seed(1)
    x = torch.randn(5, 64, 40)
    gm, bt, a = 1 + 0.1 * torch.randn(64), 0.1 * torch.randn(64), torch.rand(64) * 0.3 + 0.2
    res = torch.randn_like(x)
    y = F.group_norm(x, 4, gm, bt, 1e-5)
    want = y + (1 / a[None, :, None]) * torch.sin(a[None, :, None] * y) ** 2 + res
    got = ops.group_norm_snake(x.to(cuda), 4, gm.to(cuda), bt.to(cuda), a.to(cuda),
                               residual=res.to(cuda)).cpu()
    assert torch.allclose(got, want, atol=1e-5, rtol=1e-5)
    for shape in [(3, 8, 100), (2, 64, 300)]:  # register-cached (n <= 512) and streamed groups
        xg = torch.randn(*shape)
        yg = F.group_norm(xg, 4, gm[:shape[1]], bt[:shape[1]], 1e-5)
        ag = a[None, :shape[1], None]
        wg = yg + (1 / ag) * torch.sin(ag * yg) ** 2
        gg = ops.group_norm_snake(xg.to(cuda), 4, gm[:shape[1]].to(cuda), bt[:shape[1]].to(cuda),
                                  a[:shape[1]].to(cuda)).cpu()
        assert torch.allclose(gg, wg, atol=1e-5, rtol=1e-5), shape
    g = torch.randn(1, 64, 1)
    got = ops.channel_layernorm(x.to(cuda), g.to(cuda), residual=res.to(cuda)).cpu()
    assert torch.allclose(got, O.fe_layernorm(x, g) + res, atol=1e-5, rtol=1e-5)
    for n in (32, 301):
        qkv = torch.randn(3, 3 * 4 * 32, n)
        q, k, v = (t.reshape(3, 4, 32, n) for t in qkv.chunk(3, dim=1))
        ql, kl = q.softmax(-2) * 32 ** -0.5, k.softmax(-1)
        ctx = torch.einsum("bhdn,bhen->bhde", kl, v)
        want = torch.einsum("bhde,bhdn->bhen", ctx, ql).reshape(3, 128, n)
        got = ops.linear_attention(qkv.to(cuda), 4, 32).cpu()
        assert torch.allclose(got, want, atol=1e-5, rtol=1e-4), n
        # fused to_qkv: bitwise equal to the 1x1 conv followed by the core
        for C in (8, 24, 64):
            xin, wq = torch.randn(3, C, n).to(cuda), torch.randn(384, C, 1).to(cuda)
            unfused = ops.linear_attention(ops.conv1d(xin, wq), 4, 32)
            assert torch.equal(ops.linear_attention_fused(xin, wq, 4, 32), unfused), (n, C)
        attn = torch.einsum("bhdi,bhdj->bhij", q * 32 ** -0.5, k).softmax(-1)
        want = torch.einsum("bhij,bhdj->bhid", attn, v).permute(0, 1, 3, 2).reshape(3, 128, n)
        got = ops.attention(qkv.to(cuda), 4, 32).cpu()
        assert torch.allclose(got, want, atol=1e-5, rtol=1e-4), n
    a2, b2 = torch.randn(2, 3, 17), torch.randn(2, 5, 40)
    want = torch.cat((F.interpolate(a2, size=33, mode="linear", align_corners=False),
                      F.interpolate(b2, size=33, mode="linear", align_corners=False)), 1)
    got = ops.cat_interp(a2.to(cuda), b2.to(cuda), 33).cpu()
    assert torch.allclose(got, want, atol=1e-6, rtol=1e-6)


def _sampler(tmp_path, device):
    """TrainedModelSampler from a stage2 checkpoint (test_checkpoint's builder) and a
    Lightning-shaped stage3.ckpt holding `fidelity_enhancer.*` (sampler.py:94-106)."""
    from test_checkpoint import _build_stage2, _stage2_cfg
    from timevqvae.generation import TrainedModelSampler
    cfg = _stage2_cfg()
    cfg["fidelity_enhancer"] = dict(CFG["fidelity_enhancer"])
    s2, p1 = _build_stage2(tmp_path, cfg)
    p2, p3 = tmp_path / "stage2.ckpt", tmp_path / "stage3.ckpt"
    torch.save({"state_dict": s2.state_dict()}, p2)
    fe = _model(6, 64, 4)
    torch.save({"state_dict": {f"fidelity_enhancer.{k}": v for k, v in fe.state_dict().items()}},
               p3)
    smp = TrainedModelSampler(str(p1), str(p2), str(p3), None, input_length=64, in_channels=6,
                              n_classes=5, batch_size=16, device=device, config=cfg,
                              do_evaluate=False)
    return smp, fe


def test_sampler_loads_stage3_fidelity_enhancer(tmp_path):
    smp, fe = _sampler(tmp_path, "cpu")
    got = smp.fidelity_enhancer.state_dict()
    for k, v in fe.state_dict().items():
        assert torch.equal(got[k], v), k
    assert not smp.fidelity_enhancer.training


def test_sampler_evaluation_half_is_refused():
    from timevqvae.generation import TrainedModelSampler
    with pytest.raises(NotImplementedError):
        TrainedModelSampler(None, None, None, None, 64, 6, 5, 16, do_evaluate=True)


@pytest.mark.gpu
def test_sampler_sample_applies_fidelity_enhancer(tmp_path, cuda):
    smp, _ = _sampler(tmp_path, cuda)
    torch.manual_seed(0)
    (x_l, x_h, x), x_r = smp.sample(40, "conditional", class_index=2)
    assert x.shape == (40, 6, 64) and x_r.shape == (40, 6, 64)
    assert torch.allclose(x, x_l + x_h)
    want = torch.cat([smp.fidelity_enhancer(x[i:i + 16].to(cuda)).cpu() for i in range(0, 40, 16)])
    assert torch.equal(x_r, want)
    sd = {k: v.detach().cpu() for k, v in smp.fidelity_enhancer.state_dict().items()}
    ok, err = _close(x_r[:8].numpy(), O.fe_forward(sd, x[:8], 64).numpy())
    assert ok, err
