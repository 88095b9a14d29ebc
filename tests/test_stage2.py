"""Stage2 (MaskGIT prior): HIP transformer ops vs torch CPU fp32, the whole
BidirectionalTransformer vs the oracle restatement of x-transformers (PARITY
UNPINNED by the reference: x-transformers is absent), on-device masking vs the
oracle that is pinned to the reference's own _randomly_mask_tokens output (G5)."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import golden
from oracle import tvq_oracle as O


def rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).norm() / (b.norm() + 1e-30))


# ----------------------------------------------------------------------------- CPU
def test_oracle_mask_tokens_matches_reference():
    """oracle.random_mask_tokens reproduces maskgit.py:194-216 given the same draws."""
    g = golden("g5_maskgit.npz")
    np.random.seed(11)
    ratio = np.random.uniform(0, 1, (32,))
    torch.manual_seed(12)
    rand = torch.rand((32, 24))
    s = torch.from_numpy(g["mask_s"])
    s_M, mask = O.random_mask_tokens(s, int(g["K"]), ratio, rand)
    assert (s_M.numpy() == g["mask_s_M"]).all()
    assert (mask.numpy() == g["mask_mask"]).all()


def test_oracle_decode_loop_matches_reference():
    """A torch-RNG-faithful restatement of first_pass/second_pass reproduces the
    reference's iterative_decoding on a table-lookup stub transformer (G5)."""
    g = golden("g5_maskgit.npz")
    K = int(g["K"])
    tab_l, tab_h, tab_hl = (torch.from_numpy(g[k]) for k in ("tab_l", "tab_h", "tab_hl"))
    tf_l = lambda s_l: tab_l[torch.arange(6)[None, :], s_l]
    tf_h = lambda s_l, s_h: tab_h[torch.arange(12)[None, :], s_h] + tab_hl[s_l].mean(1, keepdim=True)
    torch.manual_seed(5)
    s_l, s_h = O.iterative_decoding_torch(tf_l, tf_h, 8, 6, 12, K, K, {"lf": 10, "hf": 1}, 10.0, 4.0)
    assert (s_l.numpy() == g["dec_s_l"]).all()
    assert (s_h.numpy() == g["dec_s_h"]).all()


# ----------------------------------------------------------------------------- GPU
def _both(shapes, cuda, seed=0, scale=1.0):
    gen = torch.Generator().manual_seed(seed)
    c = [(torch.randn(s, generator=gen) * scale).requires_grad_(True) for s in shapes]
    d = [t.detach().to(cuda).requires_grad_(True) for t in c]
    return c, d


@pytest.mark.gpu
def test_rmsnorm_layernorm(cuda):
    from timevqvae.hip.xf import layer_norm, rmsnorm
    (x, g, b), (xd, gd, bd) = _both([(300, 128), (128,), (128,)], cuda)
    yc = O.xf_rmsnorm(x, g)
    yd = rmsnorm(xd, gd)
    gy = torch.randn(yc.shape)
    yc.backward(gy); yd.backward(gy.to(cuda))
    assert rel(yd, yc) < 1e-5 and rel(xd.grad, x.grad) < 1e-5 and rel(gd.grad, g.grad) < 1e-5
    for t in (x, g, b, xd, gd, bd):
        t.grad = None
    yc = F.layer_norm(x, (128,), g, b, 1e-12)
    yd = layer_norm(xd, gd, bd, 1e-12)
    yc.backward(gy); yd.backward(gy.to(cuda))
    assert rel(yd, yc) < 1e-5 and rel(xd.grad, x.grad) < 2e-5
    assert rel(gd.grad, g.grad) < 1e-5 and rel(bd.grad, b.grad) < 1e-5


def _hash_uniform(seed, offset, ctr):
    """tvq_common.h mix_seed / uniform01 in numpy uint64 (wrapping) arithmetic."""
    u64 = np.uint64
    with np.errstate(over="ignore"):
        s = (u64(seed) * u64(0x9E3779B97F4A7C15)) ^ (u64(offset) * u64(0xC2B2AE3D27D4EB4F)
                                                    + u64(0x165667B19E3779F9))
        x = s * u64(0xD1B54A32D192ED03) + ctr.astype(np.uint64)
        x = x + u64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> u64(30))) * u64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> u64(27))) * u64(0x94D049BB133111EB)
        x = x ^ (x >> u64(31))
    return ((x >> u64(32)).astype(np.uint32) >> np.uint32(8)).astype(np.float64) / 16777216.0


@pytest.mark.gpu
@pytest.mark.parametrize("B,S,H", [(3, 25, 2), (2, 97, 1)])
def test_attention_dropout_matches_hash_mask(B, S, H, cuda):
    """Attention dropout: forward and backward both apply the documented counter-hash mask
    keep(q, k) = U(seed, offset, (bh*S + q)*S + k) >= p, scaled by 1/(1-p)."""
    from timevqvae.hip import rng
    from timevqvae.hip.xf import attention
    p, site = 0.3, 77 << 40
    (q, k, v), (qd, kd, vd) = _both([(B, S, H * 64)] * 3, cuda, seed=9)
    seed = int(rng.seed_tensor(cuda).item())
    offset = (site + rng._calls[0] + 1) & 0xFFFFFFFFFFFFFFFF
    od = attention(qd, kd, vd, H, drop_p=p, site=site)
    ctr = np.arange(B * H * S * S, dtype=np.uint64)
    keep = torch.from_numpy(_hash_uniform(seed, offset, ctr) >= p).reshape(B, H, S, S)
    sh = lambda t: t.view(B, S, H, 64).transpose(1, 2)
    a = torch.softmax(sh(q) @ sh(k).transpose(-1, -2) / 8.0, -1) * keep / (1 - p)
    oc = (a @ sh(v)).transpose(1, 2).reshape(B, S, H * 64)
    assert rel(od, oc) < 1e-5
    go = torch.randn(oc.shape)
    oc.backward(go)
    od.backward(go.to(cuda))
    for x, y in ((qd, q), (kd, k), (vd, v)):
        assert rel(x.grad, y.grad) < 2e-5


@pytest.mark.gpu
@pytest.mark.parametrize("B,S,H", [(8, 25, 2), (4, 97, 1), (2, 104, 2), (3, 1, 1), (2, 128, 1),
                                   (3, 64, 2), (5, 33, 1), (2, 96, 3)])
def test_attention(B, S, H, cuda):
    from timevqvae.hip.xf import attention
    (q, k, v), (qd, kd, vd) = _both([(B, S, H * 64)] * 3, cuda)

    def ref(q, k, v):
        sh = lambda t: t.view(B, S, H, 64).transpose(1, 2)
        a = torch.softmax(sh(q) @ sh(k).transpose(-1, -2) / 8.0, -1)
        return (a @ sh(v)).transpose(1, 2).reshape(B, S, H * 64)

    oc = ref(q, k, v)
    od = attention(qd, kd, vd, H)
    go = torch.randn(oc.shape)
    oc.backward(go); od.backward(go.to(cuda))
    assert rel(od, oc) < 1e-5
    for a, b_ in ((qd, q), (kd, k), (vd, v)):
        # S=1: softmax over one key -> dQ = dK = 0 exactly; compare with an absolute floor
        err = float((a.grad.cpu() - b_.grad).norm())
        assert err <= 2e-5 * float(b_.grad.norm()) + 1e-5 * float(go.norm()), err


@pytest.mark.gpu
def test_attention_dropout_consistent(cuda):
    """Dropout mask in fwd and bwd agree: grad equals autograd of the realised map."""
    from timevqvae.hip.xf import attention
    B, S, H = 4, 25, 2
    (q, k, v), (qd, kd, vd) = _both([(B, S, H * 64)] * 3, cuda, seed=3)
    o1 = attention(qd, kd, vd, H, drop_p=0.3, site=77)
    o0 = attention(qd.detach(), kd.detach(), vd.detach(), H)
    assert not torch.allclose(o1, o0)
    go = torch.randn_like(o1)
    o1.backward(go)
    # dropout keeps ~70% of the probability mass per row on average
    assert 0.5 < float(o1.norm() / o0.norm()) < 2.0
    assert torch.isfinite(qd.grad).all() and torch.isfinite(vd.grad).all()


@pytest.mark.gpu
def test_embedding_and_ce(cuda):
    from timevqvae.hip.xf import embedding, masked_cross_entropy
    gen = torch.Generator().manual_seed(4)
    V, D, M = 33, 128, 500
    idx = torch.randint(0, V, (M,), generator=gen)
    (tab,), (tabd,) = _both([(V, D)], cuda)
    ec = F.embedding(idx, tab)
    ed = embedding(idx.to(cuda), tabd)
    g = torch.randn(ec.shape, generator=gen)
    ec.backward(g); ed.backward(g.to(cuda))
    assert rel(ed, ec) == 0.0 and rel(tabd.grad, tab.grad) < 1e-6
    (lg,), (lgd,) = _both([(8, 24, 512)], cuda, seed=5, scale=3.0)
    tgt = torch.randint(0, 512, (8, 24), generator=gen)
    keep = torch.rand(8, 24, generator=gen) > 0.4
    lc = O.masked_ce(lg, tgt, keep)
    ld = masked_cross_entropy(lgd, tgt.to(cuda), keep.to(cuda))
    lc.backward(); ld.backward()
    assert abs(float(ld) - float(lc)) < 1e-5 * abs(float(lc))
    assert rel(lgd.grad, lg.grad) < 1e-5


@pytest.mark.gpu
def test_mask_tokens_matches_oracle(cuda):
    from timevqvae.hip.xf import mask_tokens
    gen = torch.Generator().manual_seed(6)
    for n in (24, 96):
        s = torch.randint(0, 512, (256, n), generator=gen)
        ratio = torch.rand(256, generator=gen)
        rand = torch.rand(256, n, generator=gen)
        sM_c, keep_c = O.random_mask_tokens(s, 512, ratio.double().numpy(), rand)
        sM_d, keep_d = mask_tokens(s.to(cuda), 512, 1, ratio=ratio.to(cuda), rand=rand.to(cuda))
        assert torch.equal(keep_d.cpu(), keep_c)
        assert torch.equal(sM_d.cpu(), sM_c)
    # device RNG path: statistics of the cosine schedule
    s = torch.randint(0, 512, (4096, 24), generator=gen).to(cuda)
    sM, keep = mask_tokens(s, 512, 2)
    assert (~keep).any(1).all(), "at least one masked token per row"
    assert torch.equal(torch.where(keep, s, torch.full_like(s, 512)), sM)


def _xf_state(m, seed):
    sd = {}
    gen = torch.Generator().manual_seed(seed)
    for k, v in m.state_dict().items():
        if v.is_floating_point():
            if k.endswith(("running_var",)):
                sd[k] = torch.rand(v.shape, generator=gen) + 0.5
            elif k.endswith((".g", ".gamma")) or (k.startswith("pred_head.2") and k.endswith("weight")):
                sd[k] = 1.0 + 0.1 * torch.randn(v.shape, generator=gen)
            else:
                sd[k] = torch.randn(v.shape, generator=gen) * (0.5 / math.sqrt(max(v.shape[-1], 1)) if v.dim() > 1 else 0.1)
        else:
            sd[k] = v
    m.load_state_dict(sd)
    return {k: v.clone() for k, v in sd.items()}


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["lf", "hf"])
def test_bidirectional_transformer_vs_oracle(kind, cuda):
    from timevqvae.models import BidirectionalTransformer
    K = 512
    pm = dict(hidden_dim=128, n_layers=4, heads=2, ff_mult=1) if kind == "lf" else \
        dict(hidden_dim=32, n_layers=1, heads=1, ff_mult=1)
    ntok = 24 if kind == "lf" else 96
    m = BidirectionalTransformer(kind, ntok, {"lf": K, "hf": K}, 128, use_rmsnorm=True,
                                 p_unconditional=0.0, n_classes=5, model_dropout=0.0,
                                 emb_dropout=0.0, num_tokens_l=24, **pm)
    sd = _xf_state(m, 7)
    m = m.to(cuda).train()
    gen = torch.Generator().manual_seed(8)
    B = 16
    s_l = torch.randint(0, K + 1, (B, 24), generator=gen)
    s_h = torch.randint(0, K + 1, (B, 96), generator=gen)
    y = torch.randint(0, 5, (B, 1), generator=gen)
    params = {k: v.clone().requires_grad_(True) for k, v in sd.items() if v.is_floating_point()
              and not k.endswith(("running_mean", "running_var"))}
    sdo = dict(sd)
    sdo.update(params)
    ctx = O.Ctx(True)
    lc = O.transformer_forward(ctx, sdo, kind, s_l, s_h, y, K, pm["heads"], pm["n_layers"])
    ld = m(s_l.to(cuda), s_h.to(cuda) if kind == "hf" else None, class_condition=y.to(cuda))
    assert ld.shape == lc.shape == (B, ntok, K)
    assert rel(ld, lc) < 1e-4, rel(ld, lc)
    g = torch.randn(lc.shape, generator=gen)
    lc.backward(g)
    ld.backward(g.to(cuda))
    bad = []
    for k, p in m.named_parameters():
        r = params[k].grad
        if r is None:
            continue
        e = rel(p.grad, r)
        if e > 1e-4:
            bad.append((k, e))
    assert not bad, bad


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["lf", "hf"])
def test_deferred_norm_and_conv_reductions_bitwise(kind, cuda):
    """The prior's backward into a flat gradient (FusedAdamW) inside
    wgrad_deferred(this_stream_only=True) -- the RMSNorm / LayerNorm gain gradients and the
    Upscale conv weight gradients join one batched reduction at the scope's exit
    (tvq_wgrad_defer_begin_stream) -- gives bit for bit the gradients of the immediate
    reductions."""
    from timevqvae.hip.conv import wgrad_deferred
    from timevqvae.hip.optim import FusedAdamW
    from timevqvae.models import BidirectionalTransformer
    K = 512
    pm = dict(hidden_dim=128, n_layers=4, heads=2, ff_mult=1) if kind == "lf" else \
        dict(hidden_dim=32, n_layers=1, heads=1, ff_mult=1)
    m = BidirectionalTransformer(kind, 24 if kind == "lf" else 96, {"lf": K, "hf": K}, 128,
                                 use_rmsnorm=True, p_unconditional=0.0, n_classes=5,
                                 model_dropout=0.0, emb_dropout=0.0, num_tokens_l=24, **pm)
    _xf_state(m, 11)
    m = m.to(cuda).train()
    opt = FusedAdamW(m.parameters())
    gen = torch.Generator().manual_seed(12)
    B = 32
    s_l = torch.randint(0, K + 1, (B, 24), generator=gen).to(cuda)
    s_h = torch.randint(0, K + 1, (B, 96), generator=gen).to(cuda)
    y = torch.randint(0, 5, (B, 1), generator=gen).to(cuda)
    g = torch.randn((B, 24 if kind == "lf" else 96, K), generator=gen).to(cuda)
    grads = []
    for deferred in (False, True):
        opt.zero_grad()
        out = m(s_l, s_h if kind == "hf" else None, class_condition=y)
        if deferred:
            with wgrad_deferred(this_stream_only=True):
                out.backward(g)
        else:
            out.backward(g)
        torch.cuda.synchronize()
        grads.append(opt.flat_grad.clone())
    assert grads[0].abs().sum() > 0
    assert torch.equal(grads[0], grads[1])
