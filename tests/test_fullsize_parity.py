"""Parity at the benched size: B = 256, C = 6, T = 256, K = 512 with the configs/config.yaml
architecture (BASELINE configs[1] / configs[2], the shapes bench.py times), against the oracle
(tvq_oracle, torch-CPU fp32 restatement pinned by the G3 / G9 reference goldens) or torch's CPU
ops.  At this batch the kernel plans differ from the small golden shapes: the 32x32-MFMA tile
with a 16-wide K stage (16 -> 128 conv forward, 128 -> 16 data gradient), the stride-2
weight-gradient kernel walking several stages per block (spr > 1), the fused ResBlocks reducing
256 images of BN partials.  Every test records the library's dispatch trace
(tvq_plan_trace) and asserts that the benched kernel variant is the one that ran.

Tolerances (north_star: 1e-4 relative fp32; codes index-exact):
  single ops: rel-L2 <= 1e-5 (test_ops_gpu's bar; fp32 reassociation only);
  ResBlock / whole steps: per tensor max|d - r| <= 1e-4 max|r| + 1e-6 (test_stage1's bar; a
  conv bias feeding a BatchNorm has a true gradient of 0 and is scaled by its weight's);
  code indices: equal, except rows whose fp64 top-2 distance gap is <= 1e-5 (|x|^2 +
  max|e|^2) (a near-tie that z's fp32 reassociation may flip); the oracle is then run on the
  HIP indices (tvq_oracle.Ctx.forced_ind) so the rest of the step stays comparable.
Dropout is off (p = 0) and the stage2 draws (mask ratios and scores, class drops) are
injected (maskgit.MaskGIT.forward's `draws`), as in the G3 / G9 golden tests.
"""
import contextlib
import copy

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import tvq_oracle as O

pytestmark = pytest.mark.gpu

B, C, T, K = 256, 6, 256, 512


def rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).norm() / (b.norm() + 1e-30))


def max_ok(d, r, scale=None, tol=1e-4, atol=1e-6):
    d = d.detach().double().cpu()
    r = r.detach().double().cpu()
    s = float(r.abs().max()) if scale is None else scale
    err = float((d - r).abs().max())
    return err <= tol * s + atol, err, s


def _trace():
    from timevqvae.hip._native import plan_trace
    return plan_trace()


# --------------------------------------------------------------------------- single convs
def _conv_case(kind, Ci, Co, W, cuda, want_fwd=None, want_dgrad=None, want_wgrad=None):
    """conv2d (kind 'res' 3x3 s1 zero pad, 'enc' 3x4 s(1,2) replicate) or conv_transpose2d
    ('convt' 3x4 s(1,2) p(1,1)) at B=256: output and the three gradients against torch CPU;
    the dispatch trace of each direction must contain the expected kernel."""
    from timevqvae.hip.conv import conv2d, conv_transpose2d
    gen = torch.Generator().manual_seed(Ci * 131 + Co * 7 + W)
    KH, KW = (1, 1) if kind == "proj" else (3, (3 if kind == "res" else 4))
    x = torch.randn(B, Ci, 3, W, generator=gen)
    wshape = (Ci, Co, KH, KW) if kind == "convt" else (Co, Ci, KH, KW)
    w = torch.randn(*wshape, generator=gen) * (Ci * KH * KW) ** -0.5
    b = torch.randn(Co, generator=gen) * 0.1
    xc, wc, bc = (t.clone().requires_grad_(True) for t in (x, w, b))
    if kind == "res":
        yc = F.conv2d(xc, wc, bc, padding=(1, 1))
    elif kind == "proj":
        yc = F.conv2d(xc, wc, bc)
    elif kind == "enc":
        yc = F.conv2d(F.pad(xc, (1, 1, 1, 1), mode="replicate"), wc, bc, stride=(1, 2))
    else:
        yc = F.conv_transpose2d(xc, wc, bc, stride=(1, 2), padding=(1, 1))
    g = torch.randn(yc.shape, generator=gen)
    yc.backward(g)
    xd, wd, bd = (t.to(cuda).requires_grad_(True) for t in (x, w, b))
    with _trace() as tf:
        if kind == "convt":
            yd = conv_transpose2d(xd, wd, bd)
        else:
            yd = conv2d(xd, wd, bd, stride_w=2 if kind == "enc" else 1, replicate=kind == "enc")
        torch.cuda.synchronize()
    with _trace() as tb:
        yd.backward(g.to(cuda))
        torch.cuda.synchronize()
    assert rel(yd, yc) <= 1e-5, ("fwd", rel(yd, yc))
    for n, d, c in (("dx", xd, xc), ("dw", wd, wc), ("db", bd, bc)):
        assert rel(d.grad, c.grad) <= 1e-5, (n, rel(d.grad, c.grad))
    if want_fwd:
        assert tf.has(want_fwd), (want_fwd, tf.lines)
    for want in (want_dgrad, want_wgrad):
        if want:
            assert tb.has(want), (want, tb.lines)
    return tf.lines, tb.lines


def test_conv_16_to_128_fwd_on_t32_bk16(cuda):
    """HF ResBlock(16 -> 128) first conv on (256, 16, 3, 32): forward on conv_t32 with a
    16-wide K stage (tvq_conv.hip launch_gemm, 'wide128' with bk 16)."""
    _conv_case("res", 16, 128, 32, cuda, want_fwd="conv_t32 bk16")


def test_conv_128_to_16_dgrad_on_t32_bk16(cuda):
    """HF decoder ResBlock(128 -> 16) conv on (256, 128, 3, 32): its data gradient gathers
    16 channels into 128 on the same tile."""
    _conv_case("res", 128, 16, 32, cuda, want_dgrad="conv_t32 bk16")


@pytest.mark.parametrize("kind", ["res", "proj"])
def test_conv_128_to_16_on_n16(kind, cuda):
    """HF decoder ResBlock(128 -> 16): its 3x3 conv1 and 1x1 projection forward on
    (256, 128, 3, 32) take the few-output wide-input kernel (conv_n16_kernel, one image per
    block, tap-major reduction from LDS halo planes)."""
    _conv_case(kind, 128, 16, 32, cuda, want_fwd="conv_n16 k%s mode0" % ("3x3" if kind == "res" else "1x1"))


@pytest.mark.parametrize("kind", ["res", "proj"])
def test_conv_16_to_128_dgrad_on_n16(kind, cuda):
    """HF encoder ResBlock(16 -> 128): the data gradients of its 3x3 conv1 and 1x1 projection
    (128 -> 16 gathers, flipped taps) on conv_n16_kernel."""
    _conv_case(kind, 16, 128, 32, cuda, want_dgrad="conv_n16 k%s mode1" % ("3x3" if kind == "res" else "1x1"))


# the band-end stride-2 small-channel convs at B=256 (EncBlocks: input width; ConvT: input
# width), with the stage count per block their weight gradients take (ws2_plan: <= 256 slab
# rows, so B * segments > 256 puts several 64-wide segments in one block)
S2_CASES = [("enc", 12, 4, 257, 2), ("enc", 4, 8, 128, 1), ("enc", 8, 16, 64, 1),
            ("convt", 4, 12, 128, 2), ("convt", 12, 12, 256, 4), ("convt", 8, 4, 64, 1),
            ("convt", 16, 8, 32, 1)]


@pytest.mark.parametrize("kind,Ci,Co,W,spr", S2_CASES)
def test_stride2_small_channel_convs_full_batch(kind, Ci, Co, W, spr, cuda):
    _, bwd = _conv_case(kind, Ci, Co, W, cuda, want_fwd="conv_s2",
                        want_dgrad="conv_s2t_fold" if kind == "enc" else "conv_s2f",
                        want_wgrad="conv_wgrad_s2")
    got = [int(s.split("spr=")[1]) for s in bwd if s.startswith("conv_wgrad_s2")]
    assert got == [spr], (got, bwd)


# --------------------------------------------------------------------------- fused ResBlock
def _resblock(Cc, seed, Co=None):
    from timevqvae.models.vq_vae import ResBlock
    torch.manual_seed(seed)
    m = ResBlock(Cc, Co or Cc, False, dropout=0.0)
    with torch.no_grad():
        for p in m.parameters():
            p.copy_(torch.randn_like(p) * (0.3 if p.dim() > 1 else 0.5))
        m.convs[0].a.uniform_(0.3, 0.8)
        m.convs[3].a.uniform_(0.3, 0.8)
        m.convs[2].running_mean.normal_()
        m.convs[2].running_var.uniform_(0.5, 2.0)
    return m


@pytest.mark.parametrize("Cc,W", [(8, 64), (16, 32), (32, 16), (64, 8)])
def test_fused_resblock_full_batch_vs_oracle(Cc, W, cuda):
    """ResBlock(C, C) (vq_vae.py:13-62) at the step's (256, C, 3, W) maps: the fused kernels
    (rb_fwd1/2, rb_bwd2/1; C = 64: w8_fwd1/2, w8_bwd2/1 with the image-batched weight
    gradients) against tvq_oracle.res_block with CPU autograd: output, every parameter
    gradient, dx, BN running statistics."""
    m = _resblock(Cc, 10 + Cc)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    gen = torch.Generator().manual_seed(Cc)
    x = torch.randn(B, Cc, 3, W, generator=gen) * 1.5
    gy = torch.randn(B, Cc, 3, W, generator=gen)
    # oracle
    params = {k: v.clone().requires_grad_(True) for k, v in sd.items()
              if v.is_floating_point() and not k.endswith(("running_mean", "running_var"))}
    sdo = dict(sd)
    sdo.update(params)
    xc = x.clone().requires_grad_(True)
    ctx = O.Ctx(True)
    yc = O.res_block(ctx, sdo, "", xc)
    yc.backward(gy)
    # HIP
    md = m.to(cuda).train()
    xd = x.to(cuda).requires_grad_(True)
    with _trace() as tr:
        yd = md(xd)
        yd.backward(gy.to(cuda))
        torch.cuda.synchronize()
    pre = "w8" if Cc == 64 else "rb"
    for kern in ("fwd1", "fwd2", "bwd2", "bwd1"):
        assert tr.has(f"{pre}_{kern} C{Cc} W{W} B{B}"), (kern, tr.lines)
    if Cc == 64:
        assert tr.has("conv_wgrad_w8"), tr.lines
    if Cc == 32:  # the image-batched weight gradients of both convs from the g / s planes
        assert tr.has("conv_wgrad_w16 n=2 S=16"), tr.lines
    ok, err, s = max_ok(yd, yc)
    assert ok, ("y", err, s)
    ok, err, s = max_ok(xd.grad, xc.grad)
    assert ok, ("dx", err, s)
    for k, p in md.named_parameters():
        r = params[k].grad
        scale = None
        if k == "convs.1.bias":  # feeds the BatchNorm: true gradient 0
            scale = float(params["convs.1.weight"].grad.abs().max())
        ok, err, s = max_ok(p.grad, r, scale)
        assert ok, (k, err, s)
    post = md.state_dict()
    for k, v in ctx.updates.items():
        if v.is_floating_point():
            ok, err, s = max_ok(post[k], v)
            assert ok, (k, err, s)
        else:
            assert int(post[k]) == int(v), k


@pytest.mark.parametrize("Ci,Co", [(64, 128), (128, 64)])
def test_fused_proj_resblock_full_batch_vs_oracle(Ci, Co, cuda):
    """The LF band's projection blocks ResBlock(64, 128) / ResBlock(128, 64) (vq_vae.py:13-62,
    the 1x1 proj on the skip) at the step's (256, Ci, 3, 8): w8p_fwd1/2, w8p_bwd2/1 and the
    weight gradients against tvq_oracle.res_block with CPU autograd: output, dx, every
    parameter gradient, BN running statistics."""
    m = _resblock(Ci, 7 + Ci, Co)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    gen = torch.Generator().manual_seed(Ci + Co)
    x = torch.randn(B, Ci, 3, 8, generator=gen) * 1.5
    gy = torch.randn(B, Co, 3, 8, generator=gen)
    params = {k: v.clone().requires_grad_(True) for k, v in sd.items()
              if v.is_floating_point() and not k.endswith(("running_mean", "running_var"))}
    sdo = dict(sd)
    sdo.update(params)
    xc = x.clone().requires_grad_(True)
    ctx = O.Ctx(True)
    yc = O.res_block(ctx, sdo, "", xc)
    yc.backward(gy)
    md = m.to(cuda).train()
    xd = x.to(cuda).requires_grad_(True)
    with _trace() as tr:
        yd = md(xd)
        yd.backward(gy.to(cuda))
        torch.cuda.synchronize()
    assert tr.has(f"w8p_fwd Ci{Ci} Co{Co} B{B}") and tr.has(f"w8p_bwd Ci{Ci} Co{Co} B{B}"), tr.lines
    ok, err, s = max_ok(yd, yc)
    assert ok, ("y", err, s)
    ok, err, s = max_ok(xd.grad, xc.grad)
    assert ok, ("dx", err, s)
    for k, p in md.named_parameters():
        r = params[k].grad
        scale = None
        if k == "convs.1.bias":  # feeds the BatchNorm: true gradient 0
            scale = float(params["convs.1.weight"].grad.abs().max())
        ok, err, s = max_ok(p.grad, r, scale)
        assert ok, (k, err, s)
    post = md.state_dict()
    for k, v in ctx.updates.items():
        if v.is_floating_point():
            ok, err, s = max_ok(post[k], v)
            assert ok, (k, err, s)
        else:
            assert int(post[k]) == int(v), k


# --------------------------------------------------------------------------- whole steps
def _bench_config():
    from bench import config
    cfg = config(False)
    for k in ("prior_model_l", "prior_model_h"):
        cfg["MaskGIT"][k]["model_dropout"] = 0.0
        cfg["MaskGIT"][k]["emb_dropout"] = 0.0
    return cfg


def _no_dropout(m):
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0


def _batch():
    from bench import synthetic_batch
    return synthetic_batch(1234, "cpu")


def ref_expr_flips(z, embed, got, what):
    """Code indices against the reference's own expression on the SAME z (vq.py:210-222,
    EuclideanCodebook.forward: dist = -(|x|^2 - 2 x E^T + |E|^2), argmax; fp32 torch on the
    CPU, as the reference runs it) and against its fp64 argmax: the number of rows whose HIP
    index differs, printed (the GPU test log's `flips=` lines) and returned.  A flip could
    only come from a near-tie inside fp32 rounding; the assertion is that none occurs."""
    D = embed.shape[-1]
    x = z.detach().reshape(-1, D).float().cpu()
    e = embed.detach().float().cpu().t()
    dist = -(x.pow(2).sum(1, keepdim=True) - 2 * x @ e + e.pow(2).sum(0, keepdim=True))
    ref32 = dist.argmax(-1)
    xd, ed = x.double(), e.double()
    ref64 = (-(xd.pow(2).sum(1, keepdim=True) - 2 * xd @ ed + ed.pow(2).sum(0, keepdim=True))).argmax(-1)
    g = got.detach().reshape(-1).cpu().long()
    f32, f64 = int((g != ref32).sum()), int((g != ref64).sum())
    print(f"{what}: rows={g.numel()} flips={f32} (vs the reference's fp32 torch.argmax) "
          f"flips64={f64} (vs fp64)", flush=True)
    return f32


def _check_indices(ctx, prefix):
    argmax, forced, gap, scale = ctx.ind_check[prefix]
    bad = torch.nonzero(argmax != forced).flatten()
    assert bool((gap[bad] <= 1e-5 * scale[bad]).all()), (prefix, bad[:8].tolist(), gap[bad][:8])
    return int(bad.numel())


def test_stage1_step_full_size_vs_oracle(cuda):
    """One Stage1 training step (stage1.py:89-198) at B=256 through the bench's code path
    (flat FusedAdamW gradients, pack cache, LF | HF band streams, deferred weight-gradient
    sums): the loss terms, perplexities, every parameter gradient and every buffer after the
    step (BN running statistics, VQ EMA cluster_size / embed_avg / embed) against
    tvq_oracle.stage1_forward + CPU autograd on the same weights and batch."""
    from timevqvae.hip import rng, streams
    from timevqvae.hip.conv import PackCache
    from timevqvae.trainers import Stage1
    from timevqvae.utils import set_seed
    set_seed(0)
    rng.manual_seed(1)
    s1 = Stage1(T, C, _bench_config())
    _no_dropout(s1)
    sd = {k: v.clone() for k, v in s1.state_dict().items()}
    x, y = _batch()
    s1 = s1.to(cuda).train()
    opt = s1.configure_optimizers()["optimizer"]
    s1._sched = None
    cap, zin = {}, {}
    emb0 = {n: sd[f"{n}._codebook.embed"].clone() for n in ("vq_model_l", "vq_model_h")}

    def _hook(mod, inp, o, n):
        cap[n] = o[1].detach().clone()
        zin[n] = inp[0].detach().clone()
    hooks = [getattr(s1, n).register_forward_hook(
        lambda mod, inp, o, n=n: _hook(mod, inp, o, n)) for n in ("vq_model_l", "vq_model_h")]
    opt.zero_grad()
    packs = PackCache(cuda)
    with _trace() as tr:
        with packs.scope(), streams.concurrent():
            hist = s1.forward_backward((x.to(cuda), y.to(cuda)), 0)
        out = hist()
        torch.cuda.synchronize()
    for h in hooks:
        h.remove()
    # the benched variants ran
    for want in ("conv_t32 bk16", "conv_wgrad_s2", "rb_bwd1 C16 W32 B256", "rb_bwd1 C8 W64 B256",
                 "rb_bwd1 C32 W16 B256", "w8_bwd1 C64 W8 B256", "w8_fwd2 C64 W8 B256",
                 "w8p_fwd Ci64 Co128 B256", "w8p_fwd Ci128 Co64 B256", "w8p_bwd Ci64 Co128 B256",
                 "w8p_bwd Ci128 Co64 B256", "vq_assign D128 rg6", "conv_wgrad_t32",
                 "conv_wgrad_w8"):
        assert tr.has(want), (want, sorted(set(tr.lines)))
    assert any(int(s.split("spr=")[1]) > 1 for s in tr.has("conv_wgrad_s2")), tr.has("conv_wgrad_s2")
    # oracle on the same weights, batch and (near-tie-checked) indices
    params = {k: sd[k].clone().requires_grad_(True) for k, _ in s1.named_parameters()}
    sdo = dict(sd)
    sdo.update(params)
    ctx = O.Ctx(True)
    ctx.forced_ind = {"vq_model_l.": cap["vq_model_l"].cpu(), "vq_model_h.": cap["vq_model_h"].cpu()}
    spec = O.Stage1Spec(T, C)
    ref = O.stage1_forward(ctx, sdo, spec, x)
    ref["loss"].backward()
    # index exactness: the HIP codes against the reference's own fp32 expression on the same z
    flips = {n: ref_expr_flips(zin[n], emb0[n], cap[n], f"stage1 B=256 {n}")
             for n in ("vq_model_l", "vq_model_h")}
    assert all(v == 0 for v in flips.values()), flips
    flips_oracle = sum(_check_indices(ctx, p) for p in ("vq_model_l.", "vq_model_h."))
    assert flips_oracle <= 8, flips_oracle
    for k, rk in (("loss", "loss"), ("recons_loss.LF.time", "recons_lf"),
                  ("recons_loss.HF.time", "recons_hf"), ("commit_loss.LF", "commit_lf"),
                  ("commit_loss.HF", "commit_hf"), ("perplexity.LF", "perp_lf"),
                  ("perplexity.HF", "perp_hf")):
        v, r = float(out[k].detach().sum()), float(ref[rk].detach())
        assert abs(v - r) <= 1e-4 * abs(r) + 1e-7, (k, v, r)
    bad = []
    for k, p in s1.named_parameters():
        r = params[k].grad
        scale = None
        wk = k[: -len("bias")] + "weight"
        if k.endswith(".bias") and wk in params and params[wk].dim() >= 3:
            scale = max(float(r.abs().max()), float(params[wk].grad.abs().max()))
        ok, err, s = max_ok(p.grad, r, scale)
        if not ok:
            bad.append((k, err, s))
    assert not bad, bad[:6]
    post = s1.state_dict()
    badb = []
    for k, v in ctx.updates.items():
        d = post[k].detach().cpu()
        if not v.is_floating_point():
            if not torch.equal(d, v.to(d.dtype)):
                badb.append((k, "int"))
            continue
        if k.endswith("embed"):
            err = float(((d.double() - v.double()).abs() / v.double().norm(dim=-1, keepdim=True)).max())
        else:
            err = float((d.double() - v.double()).abs().max() / (v.double().abs().max() + 1e-12))
        if err > 1e-4:
            badb.append((k, err))
    assert not badb, badb[:6]


def test_stage2_step_full_size_vs_oracle(cuda):
    """One Stage2 training step (maskgit.py:155-192, bidirectional_transformer.py:166-236)
    at B=256 with the bench's priors (LF: 4 layers, dim 128, 2 heads; HF: 1 layer, dim 32)
    through the bench's code path (flat FusedAdamW gradients, HF prior on a side stream,
    grouped Linear weight gradients), every random draw injected: tokens of the frozen
    stage1, both masked-CE losses, every gradient of both priors and the Upscale BN
    statistics against tvq_oracle.transformer_forward + masked_ce with CPU autograd."""
    from timevqvae.hip import rng, streams, wgrad
    from timevqvae.hip.conv import PackCache, wgrad_deferred
    from timevqvae.trainers import Stage1, Stage2
    from timevqvae.utils import set_seed
    set_seed(0)
    rng.manual_seed(1)
    cfg = _bench_config()
    s1 = Stage1(T, C, cfg)
    sd1 = {k: v.clone() for k, v in s1.state_dict().items()}
    s2 = Stage2(None, None, T, C, 5, config=cfg, stage1=copy.deepcopy(s1))
    mg = s2.maskgit
    sdl = {k: v.clone() for k, v in mg.transformer_l.state_dict().items()}
    sdh = {k: v.clone() for k, v in mg.transformer_h.state_dict().items()}
    x, y = _batch()
    s2 = s2.to(cuda).train()
    opt = s2.configure_optimizers()["optimizer"]
    s2._sched = None
    nl, nh = mg.num_tokens_l, mg.num_tokens_h
    g = torch.Generator().manual_seed(99)
    npr = np.random.default_rng(5)
    draws = {"ratio_l": npr.uniform(0, 1, B), "rand_l": torch.rand(B, nl, generator=g),
             "ratio_h": npr.uniform(0, 1, B), "rand_h": torch.rand(B, nh, generator=g),
             "cls_l": torch.rand(B, 1, generator=g), "cls_h": torch.rand(B, 1, generator=g)}
    xd, yd = x.to(cuda), y.to(cuda)
    from timevqvae.models import VectorQuantize
    zin = {}
    vqs = [(n, m) for n, m in mg.named_modules() if isinstance(m, VectorQuantize)]
    hooks = [m.register_forward_hook(lambda mod, inp, o, n=n: zin.__setitem__(n, (inp[0].detach().clone(), o[1].detach().clone())))
             for n, m in vqs]
    with torch.no_grad():
        s_l, s_h = mg.encode_tokens(xd)
    for h in hooks:
        h.remove()
    # index exactness of the frozen stage1's codes (encode_to_z_q, maskgit.py:94-110)
    flips = {n: ref_expr_flips(z, m._codebook.embed, ind, f"stage2 encode B=256 {n}")
             for n, m in vqs for z, ind in [zin[n]]}
    assert len(flips) == 2 and all(v == 0 for v in flips.values()), flips
    opt.zero_grad()
    packs = PackCache(cuda)
    one = torch.ones((), device=cuda)
    with _trace() as tr:
        with packs.scope(), streams.concurrent():
            loss, (loss_l, loss_h) = mg(xd, yd, draws=draws)
            with wgrad_deferred(this_stream_only=True), wgrad.grouped():
                loss.backward(one)
        torch.cuda.synchronize()
    assert tr.has("vq_assign D128"), tr.lines
    assert tr.has("w8_eval C64 W8 B256 packed=1"), tr.lines  # the frozen LF encoder
    assert tr.has("w8p_eval Ci64 Co128 B256 packed=1"), tr.lines
    assert tr.has("attn_branch_fwd B256 S25") and tr.has("attn_branch_bwd B256 S25"), tr.lines
    # tokens: the frozen stage1 (eval) through the oracle, near-ties checked
    e = O.Ctx(False)
    spec = O.Stage1Spec(T, C)
    toks = {}
    for band, enc, bandf, s in (("l", spec.enc_l, O.band_lf, s_l), ("h", spec.enc_h, O.band_hf, s_h)):
        with torch.no_grad():
            z = O.encoder_forward(e, sd1, f"encoder_{band}.", x, enc, bandf)
            e.forced_ind[f"vq_model_{band}."] = s.cpu()
            O.quantize(e, sd1, f"vq_model_{band}.", z)
        assert _check_indices(e, f"vq_model_{band}.") <= 8
        toks[band] = s.cpu()
    # oracle forward + backward with the same draws
    sM_l, keep_l = O.random_mask_tokens(toks["l"], K, draws["ratio_l"], draws["rand_l"])
    sM_h, keep_h = O.random_mask_tokens(toks["h"], K, draws["ratio_h"], draws["rand_h"])
    uncond = torch.full_like(y, 5)
    cls_l = torch.where(draws["cls_l"] > 0.2, y, uncond)
    cls_h = torch.where(draws["cls_h"] > 0.2, y, uncond)
    pl = cfg["MaskGIT"]["prior_model_l"]
    ph = cfg["MaskGIT"]["prior_model_h"]
    outs = {}
    for kind, sd, sM_args, cls, s_true, keep, pm in (
            ("lf", sdl, (sM_l, None), cls_l, toks["l"], keep_l, pl),
            ("hf", sdh, (sM_l, sM_h), cls_h, toks["h"], keep_h, ph)):
        params = {k: v.clone().requires_grad_(True) for k, v in sd.items()
                  if v.is_floating_point() and not k.endswith(("running_mean", "running_var"))}
        sdo = dict(sd)
        sdo.update(params)
        ctx = O.Ctx(True)
        logits = O.transformer_forward(ctx, sdo, kind, *sM_args, cls, K, pm["heads"], pm["n_layers"])
        lo = O.masked_ce(logits, s_true, keep)
        lo.backward()
        outs[kind] = (float(lo.detach()), params, ctx)
    for v, kind in ((loss_l, "lf"), (loss_h, "hf")):
        r = outs[kind][0]
        assert abs(float(v) - r) <= 1e-4 * abs(r), (kind, float(v), r)
    bad = []
    for kind, mod in (("lf", mg.transformer_l), ("hf", mg.transformer_h)):
        params = outs[kind][1]
        for k, p in mod.named_parameters():
            ok, err, s = max_ok(p.grad, params[k].grad, atol=1e-7)
            if not ok:
                bad.append((kind, k, err, s))
    assert not bad, bad[:6]
    post = mg.transformer_h.state_dict()
    for k, v in outs["hf"][2].updates.items():
        if k.endswith(("running_mean", "running_var")):
            assert rel(post[k], v) < 1e-5, k


@pytest.mark.parametrize("fused_ce", [False, True])
def test_stage2_per_prior_backward_roots_bitwise(fused_ce, cuda, monkeypatch):
    """MaskGIT.forward_backward (each prior backpropagated from its own loss on its own
    stream, the bench's stage2 path) gives bit for bit the gradients and losses of
    forward() + loss.backward() on the same draws (B = 256, the bench's priors, layer dropout
    on the device seed, reset between the two runs) -- with the loss heads unfused.  With the
    fused loss head (tied_logits_ce: the logits, the masked CE and dlogits / dh in one pass,
    the default of forward_backward) the sums run in another order: the flat gradient within
    1e-4 of its largest entry's magnitude per parameter segment, the losses within 1e-5."""
    from timevqvae.hip import rng, streams, wgrad
    from timevqvae.models import bidirectional_transformer as bt
    monkeypatch.setattr(bt, "TIED_CE_FUSED", fused_ce)
    from timevqvae.hip.conv import PackCache, wgrad_deferred
    from timevqvae.trainers import Stage1, Stage2
    from timevqvae.utils import set_seed
    set_seed(0)
    cfg = _bench_config()
    s1 = Stage1(T, C, cfg)
    s2 = Stage2(None, None, T, C, 5, config=cfg, stage1=copy.deepcopy(s1)).to(cuda).train()
    mg = s2.maskgit
    opt = s2.configure_optimizers()["optimizer"]
    s2._sched = None
    nl, nh = mg.num_tokens_l, mg.num_tokens_h
    g = torch.Generator().manual_seed(7)
    npr = np.random.default_rng(3)
    draws = {"ratio_l": npr.uniform(0, 1, B), "rand_l": torch.rand(B, nl, generator=g),
             "ratio_h": npr.uniform(0, 1, B), "rand_h": torch.rand(B, nh, generator=g),
             "cls_l": torch.rand(B, 1, generator=g), "cls_h": torch.rand(B, 1, generator=g)}
    x, y = _batch()
    xd, yd = x.to(cuda), y.to(cuda)
    one = torch.ones((), device=cuda)
    packs = PackCache(cuda)
    res = []
    for split in (False, True):
        rng.manual_seed(11)
        rng.restart_calls()
        opt.zero_grad()
        with packs.scope(), streams.concurrent():
            with wgrad_deferred(this_stream_only=True), wgrad.grouped():
                if split:
                    total = mg.forward_backward(xd, yd, one, draws=draws)
                else:
                    loss, parts = mg(xd, yd, draws=draws)
                    loss.backward(one)
        if split:
            loss, parts = total()
        torch.cuda.synchronize()
        res.append((opt.flat_grad.clone(), float(loss), [float(p) for p in parts]))
    assert res[0][0].abs().sum() > 0
    if not fused_ce:
        assert torch.equal(res[0][0], res[1][0])
        assert res[0][1] == res[1][1] and res[0][2] == res[1][2]
        return
    g0, g1 = res[0][0].double(), res[1][0].double()
    off = 0  # the flat gradient holds the parameters in param-group order
    for p in (q for grp in opt.param_groups for q in grp["params"]):
        n = p.numel()
        a, b = g1[off:off + n], g0[off:off + n]
        off += n
        if b.abs().max() > 0:
            assert float((a - b).abs().max() / b.abs().max()) < 1e-4, tuple(p.shape)
    assert abs(res[0][1] - res[1][1]) <= 1e-5 * abs(res[0][1])
    for a, b in zip(res[1][2], res[0][2]):
        assert abs(a - b) <= 1e-5 * abs(b)
