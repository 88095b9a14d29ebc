"""Stage2 pinned to the reference's own files (G9, tests/golden/make_golden.py:gen_stage2).

G9 ran reference bidirectional_transformer.py (Upscale, embeddings, class conditioning,
pred_head, tied logits) and maskgit.py (forward loss composition, masking, CFG) with
x-transformers replaced by the T1 restatement (the package is absent: its arithmetic
alone stays parity-unpinned).  Every random draw of the reference (np ratios, torch.rand
masking scores, class-drop draws) was recorded, so the HIP path is fed the same draws.

Tolerances: logits / losses rel-norm <= 1e-4 (north_star's fp32 bar); gradients per
tensor |g - g_ref|max <= 1e-4 * max|g_ref| + 1e-7; token indices bit-exact.
"""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import tvq_oracle as O
from param_init import fill_state_dict

K = 512
PRIOR = {"lf": dict(hidden_dim=128, n_layers=4, heads=2, ff_mult=1, use_rmsnorm=True),
         "hf": dict(hidden_dim=32, n_layers=1, heads=1, ff_mult=1, use_rmsnorm=True)}
SEED = {"lf": 41, "hf": 42}


def gout(shape, seed):
    # make_golden.gout: the upstream gradient of the G9 backward checks
    return np.random.default_rng(seed + 200).standard_normal(shape).astype(np.float32)


def rel(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.linalg.norm(a - b) / (np.linalg.norm(b) + 1e-30))


def build_transformer(kind, Kc=K, emb=128, seed=None, ntok=None, ntok_l=24):
    from timevqvae.models import BidirectionalTransformer
    ntok = ntok if ntok is not None else (24 if kind == "lf" else 96)
    m = BidirectionalTransformer(kind, ntok, {"lf": Kc, "hf": Kc}, emb, p_unconditional=0.2,
                                 n_classes=5, model_dropout=0.0, emb_dropout=0.0,
                                 num_tokens_l=ntok_l, **PRIOR[kind])
    sd = m.state_dict()
    vals = fill_state_dict(sd, SEED[kind] if seed is None else seed)
    sd.update({k: torch.from_numpy(v) for k, v in vals.items()})
    m.load_state_dict(sd, strict=True)
    return m, {k: v.clone() for k, v in sd.items()}


def grads_ok(named, ref, prefix):
    bad = []
    for k, g in named:
        r = ref[prefix + k]
        d = g.detach().cpu().numpy()
        if np.abs(d - r).max() > 1e-4 * np.abs(r).max() + 1e-7:
            bad.append((k, float(np.abs(d - r).max()), float(np.abs(r).max())))
    return bad


# ----------------------------------------------------------------------------- CPU
@pytest.mark.parametrize("kind", ["lf", "hf"])
def test_transformer_state_dict_keys_match_reference(kind):
    """Module tree (and so checkpoint keys) equals the reference file's, x-transformers
    layout included (bidirectional_transformer.py:34-122)."""
    g = golden("g9_stage2.npz")
    m, _ = build_transformer(kind)
    assert sorted(m.state_dict().keys()) == sorted(g[f"{kind}_keys"].tolist())


@pytest.mark.parametrize("kind", ["lf", "hf"])
def test_oracle_transformer_matches_reference(kind):
    """The oracle's forward_lf/forward_hf restatement equals the reference file's output
    (eval with and without class, train-mode with the recorded class-drop draws) and its
    gradients: pins T0 Upscale, T2 and the tied logits of the oracle."""
    g = golden("g9_stage2.npz")
    _, sd = build_transformer(kind)
    p = kind + "_"
    s_l, s_h, y = (torch.from_numpy(g[p + k]) for k in ("s_l", "s_h", "y"))
    pm = PRIOR[kind]
    for key, cls in (("eval_cond", y), ("eval_uncond", torch.full_like(y, 5))):
        with torch.no_grad():
            lc = O.transformer_forward(O.Ctx(False), sd, kind, s_l, s_h, cls, K, pm["heads"],
                                       pm["n_layers"])
        assert rel(lc.numpy(), g[p + key]) < 1e-5, key
    cls = torch.where(torch.from_numpy(g[p + "train_cls_rand"]) > 0.2, y, torch.full_like(y, 5))
    params = {k: v.clone().requires_grad_(True) for k, v in sd.items()
              if v.is_floating_point() and not k.endswith(("running_mean", "running_var"))}
    sdo = dict(sd)
    sdo.update(params)
    ctx = O.Ctx(True)
    lc = O.transformer_forward(ctx, sdo, kind, s_l, s_h, cls, K, pm["heads"], pm["n_layers"])
    assert rel(lc.detach().numpy(), g[p + "train_cond"]) < 1e-5
    (lc * torch.from_numpy(gout(lc.shape, SEED[kind]))).sum().backward()
    bad = grads_ok(((k, v.grad) for k, v in params.items()), g, p + "grad/")
    assert not bad, bad[:5]
    for k, v in ctx.updates.items():
        if k.endswith(("running_mean", "running_var")):
            assert rel(v.numpy(), g[p + "post/" + k]) < 1e-6, k


def _maskgit_cpu_sd():
    """Stage1 (G3-small weights, seed 3) + transformers (seed 50) state, product keys."""
    from test_stage1 import make_config
    from timevqvae.trainers import Stage1
    s1 = Stage1(128, 6, make_config(64, 4, 32))
    vals = fill_state_dict(s1.state_dict(), 3)
    s1.load_state_dict({k: torch.from_numpy(v) for k, v in vals.items()}, strict=False)
    tl, sdl = build_transformer("lf", Kc=64, emb=32, seed=50)
    th, sdh = build_transformer("hf", Kc=64, emb=32, seed=50)
    return s1, tl, th, sdl, sdh


def test_oracle_maskgit_loss_matches_reference():
    """masked CE composition (maskgit.py:166-192) of the oracle with G9's recorded draws
    and the reference's own token indices equals the reference loss."""
    g = golden("g9_stage2.npz")
    _, _, _, sdl, sdh = _maskgit_cpu_sd()
    s_l, s_h = torch.from_numpy(g["mg_s_l"]), torch.from_numpy(g["mg_s_h"])
    y = torch.from_numpy(g["mg_y"])
    sM_l, keep_l = O.random_mask_tokens(s_l, 64, g["mg_ratio_l"], torch.from_numpy(g["mg_rand_l"]))
    sM_h, keep_h = O.random_mask_tokens(s_h, 64, g["mg_ratio_h"], torch.from_numpy(g["mg_rand_h"]))
    cls_l = torch.where(torch.from_numpy(g["mg_cls_rand_l"]) > 0.2, y, torch.full_like(y, 5))
    cls_h = torch.where(torch.from_numpy(g["mg_cls_rand_h"]) > 0.2, y, torch.full_like(y, 5))
    with torch.no_grad():
        ll = O.transformer_forward(O.Ctx(True), sdl, "lf", sM_l, None, cls_l, 64, 2, 4)
        lh = O.transformer_forward(O.Ctx(True), sdh, "hf", sM_l, sM_h, cls_h, 64, 1, 1)
    loss_l, loss_h = float(O.masked_ce(ll, s_l, keep_l)), float(O.masked_ce(lh, s_h, keep_h))
    assert abs(loss_l - float(g["mg_loss_l"])) < 1e-5 * abs(float(g["mg_loss_l"]))
    assert abs(loss_h - float(g["mg_loss_h"])) < 1e-5 * abs(float(g["mg_loss_h"]))


# ----------------------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["lf", "hf"])
def test_transformer_eval_logits_vs_reference(kind, cuda):
    g = golden("g9_stage2.npz")
    m, _ = build_transformer(kind)
    m = m.to(cuda).eval()
    p = kind + "_"
    s_l, s_h, y = (torch.from_numpy(g[p + k]).to(cuda) for k in ("s_l", "s_h", "y"))
    args = (s_l,) if kind == "lf" else (s_l, s_h)
    with torch.no_grad():
        lc = m(*args, class_condition=y).cpu().numpy()
        lu = m(*args, class_condition=None).cpu().numpy()
    assert rel(lc, g[p + "eval_cond"]) < 1e-4
    assert rel(lu, g[p + "eval_uncond"]) < 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["lf", "hf"])
def test_transformer_train_step_vs_reference(kind, cuda):
    """Train mode: class-drop draws injected, Upscale BN on batch statistics; logits,
    every parameter gradient and the BN running statistics against the reference."""
    g = golden("g9_stage2.npz")
    m, _ = build_transformer(kind)
    m = m.to(cuda).train()
    p = kind + "_"
    s_l, s_h, y = (torch.from_numpy(g[p + k]).to(cuda) for k in ("s_l", "s_h", "y"))
    args = (s_l,) if kind == "lf" else (s_l, s_h)
    m._class_rand = torch.from_numpy(g[p + "train_cls_rand"])
    logits = m(*args, class_condition=y)
    m._class_rand = None
    assert rel(logits.detach().cpu().numpy(), g[p + "train_cond"]) < 1e-4
    (logits * torch.from_numpy(gout(logits.shape, SEED[kind])).to(cuda)).sum().backward()
    bad = grads_ok(((k, q.grad) for k, q in m.named_parameters()), g, p + "grad/")
    assert not bad, bad[:5]
    for k, v in m.state_dict().items():
        if k.endswith(("running_mean", "running_var")):
            assert rel(v.cpu().numpy(), g[p + "post/" + k]) < 1e-5, k


def _maskgit(cuda):
    from timevqvae.models.maskgit import MaskGIT
    from test_stage1 import make_config
    s1, tl, th, _, _ = _maskgit_cpu_sd()
    cfg = make_config(64, 4, 32)
    prior = dict(p_unconditional=0.2, model_dropout=0.0, emb_dropout=0.0)
    cfg["MaskGIT"] = {"choice_temperatures": {"lf": 10, "hf": 4}, "T": {"lf": 10, "hf": 1},
                      "prior_model_l": {**PRIOR["lf"], **prior},
                      "prior_model_h": {**PRIOR["hf"], **prior}, "cfg_scale": 1.0}
    mg = MaskGIT(None, 128, 6, cfg, 5, cfg["MaskGIT"]["choice_temperatures"], cfg["MaskGIT"]["T"],
                 stage1=s1)
    mg.transformer_l.load_state_dict(tl.state_dict())
    mg.transformer_h.load_state_dict(th.state_dict())
    return mg.to(cuda)


@pytest.mark.gpu
def test_maskgit_forward_loss_vs_reference(cuda):
    """MaskGIT.forward (maskgit.py:155-192) with the reference's recorded draws: tokens
    exact, losses within 1e-4, every transformer gradient within tolerance."""
    g = golden("g9_stage2.npz")
    mg = _maskgit(cuda).train()
    x = torch.from_numpy(g["mg_x"]).to(cuda)
    y = torch.from_numpy(g["mg_y"]).to(cuda)
    s_l, s_h = mg.encode_tokens(x)
    assert np.array_equal(s_l.cpu().numpy(), g["mg_s_l"])
    assert np.array_equal(s_h.cpu().numpy(), g["mg_s_h"])
    draws = {"ratio_l": g["mg_ratio_l"], "rand_l": g["mg_rand_l"], "ratio_h": g["mg_ratio_h"],
             "rand_h": g["mg_rand_h"], "cls_l": torch.from_numpy(g["mg_cls_rand_l"]),
             "cls_h": torch.from_numpy(g["mg_cls_rand_h"])}
    loss, (loss_l, loss_h) = mg(x, y, draws=draws)
    for v, k in ((loss, "mg_loss"), (loss_l, "mg_loss_l"), (loss_h, "mg_loss_h")):
        assert abs(float(v) - float(g[k])) <= 1e-4 * abs(float(g[k])), (k, float(v), float(g[k]))
    loss.backward()
    named = [(f"{n}.{k}", q.grad) for n in ("transformer_l", "transformer_h")
             for k, q in getattr(mg, n).named_parameters()]
    bad = grads_ok(named, g, "mg_grad/")
    assert not bad, bad[:5]
    for k in g:  # the HF Upscale BatchNorm's running statistics after the forward
        if k.startswith("mg_post/"):
            name, kk = k[len("mg_post/"):].split(".", 1)
            v = getattr(mg, name).state_dict()[kk].cpu().numpy()
            assert rel(v, g[k]) < 1e-5, k


@pytest.mark.gpu
def test_masked_prediction_cfg_vs_reference(cuda):
    """Classifier-free guidance, cfg_scale 2 (maskgit.py:136-153), eval mode."""
    g = golden("g9_stage2.npz")
    mg = _maskgit(cuda).eval()
    mg.cfg_scale = 2.0
    with torch.no_grad():  # the reference ran this after its training forward (BN stats)
        for k in g:
            if k.startswith("mg_post/"):
                name, kk = k[len("mg_post/"):].split(".", 1)
                getattr(mg, name).state_dict()[kk].copy_(torch.from_numpy(g[k]))
    y = torch.from_numpy(g["mg_y"]).to(cuda)
    sl, sh = torch.from_numpy(g["cfg_s_l_M"]).to(cuda), torch.from_numpy(g["cfg_s_h_M"]).to(cuda)
    with torch.no_grad():
        ll = mg.masked_prediction(mg.transformer_l, y, sl).cpu().numpy()
        lh = mg.masked_prediction(mg.transformer_h, y, sl, sh).cpu().numpy()
        lu = mg.masked_prediction(mg.transformer_h, None, sl, sh).cpu().numpy()
    assert rel(ll, g["cfg_logits_l"]) < 1e-4
    assert rel(lh, g["cfg_logits_h"]) < 1e-4
    assert rel(lu, g["cfg_logits_h_uncond"]) < 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("tag", ["small", "cfgB", "cfgA"])
def test_encode_tokens_vs_reference(tag, cuda):
    """M1: MaskGIT's fused encode (one STFT pass, eval encoders, VQ assign) gives the
    reference's quantize() indices of G3 (encode_to_z_q, maskgit.py:117-134)."""
    from test_stage1 import _index_ok, build
    from timevqvae.models.maskgit import MaskGIT
    m, g3 = build(tag, cuda)
    mg = MaskGIT.__new__(MaskGIT)
    torch.nn.Module.__init__(mg)
    m.eval()
    mg.encoder_l, mg.encoder_h = m.encoder_l, m.encoder_h
    mg.vq_model_l, mg.vq_model_h = m.vq_model_l, m.vq_model_h
    x = torch.from_numpy(g3["x"]).to(cuda)
    s_l, s_h = MaskGIT.encode_tokens(mg, x)
    for s, zk, ik, vq in ((s_l, "eval_z_l", "eval_s_l", m.vq_model_l),
                          (s_h, "eval_z_h", "eval_s_h", m.vq_model_h)):
        z = g3[zk]
        zt = z.transpose(0, 2, 3, 1).reshape(-1, z.shape[1])
        E = vq._codebook.embed.detach().cpu().numpy()
        assert _index_ok(s.cpu().numpy(), g3[ik], zt, E), ik
