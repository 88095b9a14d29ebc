"""Generate golden input/output vectors from the REFERENCE implementation.

Runs only in the build container (it reads /root/reference, which does not
exist on the GPU box).  The reference package cannot be imported as a whole
(lightning, mlflow, x_transformers, traffic ... are absent), so the hot-path
files are loaded by file path with minimal import stubs:

  * timevqvae/models/vq.py            (torch + einops only)
  * timevqvae/utils/train_utils.py     (stub: mlflow)
  * timevqvae/models/vq_vae.py         (synthetic timevqvae.utils)
  * timevqvae/trainers/stage1.py       (stub: lightning.LightningModule = nn.Module)
  * timevqvae/models/maskgit.py        (stub transformer; sampling/masking loops only)

G6 (stochastic VQ) alone: python tests/golden/make_golden.py svq
G7 (ROCKET features, evaluation/rocket_functions.py with a numba stub) alone: ... rocket
G8 (FidelityEnhancer / Unet1D forward, models/fidelity_enhancer.py) alone: ... fe
G10 (calculate_fid, evaluation/eval_utils.py) alone: ... fid
G11 (Stage3 FE training loss + gradients, trainers/stage3.py) alone: ... fetrain

Only the .npz outputs are committed (tests/golden/*.npz).  Usage:

    python tests/golden/make_golden.py            # writes tests/golden/*.npz
"""
import importlib.util
import os
import sys
import types

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from param_init import fill_state_dict  # noqa: E402

REF = "/root/reference/timevqvae"
OUT = os.path.dirname(os.path.abspath(__file__))


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def load_reference():
    """Load the hot-path reference files with import stubs; returns a namespace."""
    # --- stubs for absent third-party packages (never executed on a hot path) ---
    mlflow = types.ModuleType("mlflow")
    mlflow.log_artifact = lambda *a, **k: None
    sys.modules.setdefault("mlflow", mlflow)
    lightning = types.ModuleType("lightning")
    lightning.LightningModule = nn.Module
    sys.modules.setdefault("lightning", lightning)

    pkg = types.ModuleType("timevqvae")
    pkg.__path__ = []
    sys.modules["timevqvae"] = pkg
    vq = _load("ref_vq", f"{REF}/models/vq.py")
    tu = _load("ref_train_utils", f"{REF}/utils/train_utils.py")
    utils = types.ModuleType("timevqvae.utils")
    for k in dir(tu):
        if not k.startswith("__"):
            setattr(utils, k, getattr(tu, k))
    sys.modules["timevqvae.utils"] = utils
    vqvae = _load("ref_vq_vae", f"{REF}/models/vq_vae.py")
    models = types.ModuleType("timevqvae.models")
    models.VectorQuantize = vq.VectorQuantize
    models.VQVAEEncoder = vqvae.VQVAEEncoder
    models.VQVAEDecoder = vqvae.VQVAEDecoder
    models.BidirectionalTransformer = object  # stub: x_transformers is absent
    sys.modules["timevqvae.models"] = models
    stage1 = _load("ref_stage1", f"{REF}/trainers/stage1.py")
    maskgit = _load("ref_maskgit", f"{REF}/models/maskgit.py")
    return types.SimpleNamespace(vq=vq, tu=tu, vqvae=vqvae, stage1=stage1, maskgit=maskgit)


def _sd(module, prefix):
    return {f"{prefix}{k}": v.detach().cpu().numpy().copy() for k, v in module.state_dict().items()}


# --------------------------------------------------------------------------- G0/G1
def gen_vq(ref):
    out = {}
    # G0: the reference's own __main__ known-answer test (vq.py:410-424)
    torch.manual_seed(0)
    x = torch.rand((1024, 32, 128))
    vqm = ref.vq.VectorQuantize(dim=128, codebook_size=512)
    q, ind, loss, perp = vqm(x)
    out["kat_ind0"] = ind[0].numpy().astype(np.int64)
    out["kat_n_unique"] = np.array(len(torch.unique(ind)))
    out["kat_commit"] = np.array(float(loss["commit_loss"]))
    out["kat_perplexity"] = np.array(float(perp))
    out["kat_cs_sum"] = np.array(float(vqm._codebook.cluster_size.sum()))
    out["kat_embed0"] = vqm._codebook.embed[0, :4].numpy().copy()
    np.savez_compressed(f"{OUT}/g0_vq_kat.npz", **out)

    # G1: full vectors, random codebook and data-near codebook, train (EMA) mode
    for variant in ("random", "near"):
        g = torch.Generator().manual_seed(1234 if variant == "random" else 4321)
        B, N, D, K = 8, 128, 128, 512  # M = 1024 rows
        x = torch.randn(B, N, D, generator=g)
        vqm = ref.vq.VectorQuantize(dim=D, codebook_size=K)
        if variant == "near":
            flat = x.reshape(-1, D)
            perm = torch.randperm(flat.shape[0], generator=g)[:K]
            E = flat[perm] + 0.05 * torch.randn(K, D, generator=g)
            vqm._codebook.embed.data.copy_(E)
            vqm._codebook.embed_avg.data.copy_(E)
        # pre-existing EMA state so the blend is exercised
        vqm._codebook.cluster_size.data.copy_(torch.rand(K, generator=g) * 3)
        d = {
            "x": x.numpy(),
            "embed": vqm._codebook.embed.numpy().copy(),
            "embed_avg": vqm._codebook.embed_avg.numpy().copy(),
            "cluster_size": vqm._codebook.cluster_size.numpy().copy(),
        }
        # eval-mode assignment first (no EMA), then one train-mode forward
        vqm.eval()
        q_e, ind_e, _, perp_e = vqm(x)
        d["eval_ind"] = ind_e.numpy().astype(np.int64)
        d["eval_perplexity"] = np.array(float(perp_e))
        vqm.train()
        xg = x.clone().requires_grad_(True)
        q, ind, loss, perp = vqm(xg)
        (q.square().sum() * 0.5 + loss["loss"].sum()).backward()
        d["ind"] = ind.numpy().astype(np.int64)
        d["commit"] = np.array(float(loss["commit_loss"]))
        d["perplexity"] = np.array(float(perp))
        d["post_cluster_size"] = vqm._codebook.cluster_size.numpy().copy()
        d["post_embed_avg"] = vqm._codebook.embed_avg.numpy().copy()
        d["post_embed"] = vqm._codebook.embed.numpy().copy()
        d["x_grad"] = xg.grad.numpy()  # d/dx [0.5*sum(q_st^2) + commit]
        # fp64 top-2 gap per row (to qualify near-ties)
        f64 = x.double().reshape(-1, D)
        E64 = torch.from_numpy(d["embed"]).double()
        dist = (f64.pow(2).sum(1, keepdim=True) - 2 * f64 @ E64.t() + E64.pow(2).sum(1)[None])
        top2 = dist.topk(2, dim=1, largest=False).values
        d["gap64"] = (top2[:, 1] - top2[:, 0]).numpy()
        np.savez_compressed(f"{OUT}/g1_vq_{variant}.npz", **d)


# --------------------------------------------------------------------------- G2
def gen_stft(ref):
    tu = ref.tu
    d = {}
    for T in (128, 256):
        g = torch.Generator().manual_seed(7 + T)
        x = torch.cumsum(0.1 * torch.randn(4, 6, T, generator=g), -1)
        xf = tu.time_to_timefreq(x, 4, 6)
        d[f"x_T{T}"] = x.numpy()
        d[f"xf_T{T}"] = xf.numpy()
        d[f"lf_copy_T{T}"] = tu.zero_pad_high_freq(xf, copy=True).numpy()
        d[f"hf_copy_T{T}"] = tu.zero_pad_low_freq(xf, copy=True).numpy()
        u_l = tu.zero_pad_high_freq(xf)
        u_h = tu.zero_pad_low_freq(xf)
        d[f"u_l_T{T}"] = u_l.numpy()
        d[f"u_h_T{T}"] = u_h.numpy()
        x_l = torch.nn.functional.interpolate(tu.timefreq_to_time(u_l, 4, 6), T, mode="linear")
        x_h = torch.nn.functional.interpolate(tu.timefreq_to_time(u_h, 4, 6), T, mode="linear")
        d[f"x_l_T{T}"] = x_l.numpy()
        d[f"x_h_T{T}"] = x_h.numpy()
        # decoder-side istft on a 2x-upsampled random image (W = 2*T frames)
        img = torch.randn(4, 12, 3, 2 * T, generator=g)
        d[f"dec_img_T{T}"] = img.numpy()
        d[f"dec_istft_lf_T{T}"] = tu.timefreq_to_time(tu.zero_pad_high_freq(img), 4, 6).numpy()
        d[f"dec_istft_hf_T{T}"] = tu.timefreq_to_time(tu.zero_pad_low_freq(img), 4, 6).numpy()
        d[f"snake_a_in_T{T}"] = img[:, :, :, :7].numpy()
    np.savez_compressed(f"{OUT}/g2_stft.npz", **d)


# --------------------------------------------------------------------------- G3/G4
def _stage1_config(init_dim, hid_dim, K):
    return {
        "VQ-VAE": {"n_fft": 4, "codebook_sizes": {"lf": K, "hf": K}},
        "encoder": {"init_dim": init_dim, "hid_dim": hid_dim, "n_resnet_blocks": 2,
                    "downsampled_width": {"lf": 8, "hf": 32}},
        "decoder": {"n_resnet_blocks": 2},
        "exp_params": {"lr": 1e-3, "linear_warmup_rate": 0.1},
        "trainer_params": {"max_steps": {"stage1": 1000, "stage2": 1000}},
    }


def gen_stage1(ref, tag, B, C, T, K, init_dim, hid_dim, seed):
    torch.manual_seed(seed)
    np.random.seed(seed)
    cfg = _stage1_config(init_dim, hid_dim, K)
    model = ref.stage1.Stage1(T, C, cfg)
    # dropout off so the train-mode step is deterministic (SURVEY §7 hard parts)
    for m in model.modules():
        if isinstance(m, nn.Dropout):
            m.p = 0.0
    g = torch.Generator().manual_seed(seed + 1)
    x = torch.cumsum(0.1 * torch.randn(B, C, T, generator=g), -1)
    x = 2 * (x - x.amin(0, keepdim=True)) / (x.amax(0, keepdim=True) - x.amin(0, keepdim=True) + 1e-8) - 1
    y = torch.randint(0, 5, (B, 1), generator=g)
    d = {"x": x.numpy(), "y": y.numpy(), "cfg": np.array([B, C, T, K, init_dim, hid_dim]),
         "seed": np.array(seed)}
    # parameters/buffers from the shared deterministic rule (param_init.py)
    vals = fill_state_dict(model.state_dict(), seed)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in vals.items()}, strict=False)

    # eval-mode reconstruction on the initial state
    model.eval()
    with torch.no_grad():
        d["eval_x_rec"] = model((x, y), 0, return_x_rec=True).numpy()
        z = model.encoder_l(x)
        d["eval_z_l"] = z.numpy()
        _, s, _, _ = ref.tu.quantize(z, model.vq_model_l)
        d["eval_s_l"] = s.numpy().astype(np.int64)
        z = model.encoder_h(x)
        d["eval_z_h"] = z.numpy()
        _, s, _, _ = ref.tu.quantize(z, model.vq_model_h)
        d["eval_s_h"] = s.numpy().astype(np.int64)

    # train-mode forward + backward (one step's gradients)
    model.train()
    cap = {}

    def hook(name):
        def f(mod, inp, out):
            if isinstance(out, tuple):
                cap[name] = out[0].detach().clone()
                cap[name + "_ind"] = out[1].detach().clone()
            else:
                cap[name] = out.detach().clone()
        return f

    for name in ("encoder_l", "encoder_h", "vq_model_l", "vq_model_h", "decoder_l", "decoder_h"):
        getattr(model, name).register_forward_hook(hook(name))
    recons, vq_losses, perps = model((x, y), 0)
    loss = recons["LF.time"] + recons["HF.time"] + vq_losses["LF"]["loss"] + vq_losses["HF"]["loss"]
    loss.backward()
    d["train_loss"] = np.array(float(loss))
    d["train_recons_lf"] = np.array(float(recons["LF.time"]))
    d["train_recons_hf"] = np.array(float(recons["HF.time"]))
    d["train_commit_lf"] = np.array(float(vq_losses["LF"]["commit_loss"]))
    d["train_commit_hf"] = np.array(float(vq_losses["HF"]["commit_loss"]))
    d["train_perp_lf"] = np.array(float(perps["LF"]))
    d["train_perp_hf"] = np.array(float(perps["HF"]))
    for k, v in cap.items():
        d[f"train_{k}"] = v.numpy()
    for k, p in model.named_parameters():
        if p.grad is not None:
            d[f"grad/{k}"] = p.grad.numpy().copy()
    d.update({f"post/{k}": v.detach().numpy().copy() for k, v in model.named_buffers()})
    np.savez_compressed(f"{OUT}/g3_stage1_{tag}.npz", **d)


# --------------------------------------------------------------------------- G5
def gen_maskgit(ref):
    MG = ref.maskgit.MaskGIT
    mg = MG.__new__(MG)
    nn.Module.__init__(mg)
    K = 16
    mg.T = {"lf": 10, "hf": 1}
    mg.mask_token_ids = {"lf": K, "hf": K}
    mg.choice_temperature_l, mg.choice_temperature_h = 10.0, 4.0
    mg.cfg_scale = 1.0
    mg.gamma = mg.gamma_func("cosine")
    mg.num_tokens_l, mg.num_tokens_h = 6, 12

    # deterministic stub transformers: logits = table lookup over (position, input token)
    gt = torch.Generator().manual_seed(99)
    tab_l = torch.randn(6, K + 1, K, generator=gt) * 2
    tab_h = torch.randn(12, K + 1, K, generator=gt) * 2
    tab_hl = torch.randn(K + 1, K, generator=gt)

    def tf_l(s_l, class_condition=None):
        return tab_l[torch.arange(6)[None, :], s_l]

    def tf_h(s_l, s_h, class_condition=None):
        return tab_h[torch.arange(12)[None, :], s_h] + tab_hl[s_l].mean(1, keepdim=True)

    mg.transformer_l, mg.transformer_h = tf_l, tf_h
    d = {"tab_l": tab_l.numpy(), "tab_h": tab_h.numpy(), "tab_hl": tab_hl.numpy(), "K": np.array(K)}
    torch.manual_seed(5)
    s_l, s_h = mg.iterative_decoding(num=8, device="cpu")
    d["dec_s_l"] = s_l.numpy().astype(np.int64)
    d["dec_s_h"] = s_h.numpy().astype(np.int64)

    # training-time masking
    np.random.seed(11)
    torch.manual_seed(12)
    s = torch.randint(0, K, (32, 24), generator=torch.Generator().manual_seed(13))
    s_M, mask = mg._randomly_mask_tokens(s, K, "cpu")
    d["mask_s"] = s.numpy().astype(np.int64)
    d["mask_s_M"] = s_M.numpy().astype(np.int64)
    d["mask_mask"] = mask.numpy()

    # mask_by_random_topk with fixed probs
    torch.manual_seed(21)
    probs = torch.rand(4, 12)
    probs[:, :3] = torch.inf
    masking = mg.mask_by_random_topk(torch.full((4, 1), 5.0), probs, temperature=3.0)
    d["topk_probs"] = probs.numpy()
    d["topk_masking"] = masking.numpy()
    np.savez_compressed(f"{OUT}/g5_maskgit.npz", **d)


# --------------------------------------------------------------------------- G6
def gen_svq(ref):
    """Stochastic VQ (svq_temp > 0): EuclideanCodebook.forward draws idx with
    softmax_sample = Categorical(logits=dist/temp).sample() (vq.py:51-56, 216-222).  The
    draws are torch's CPU RNG under the recorded seeds, so the oracle restatement
    (same logits, same sampler, same seed) must reproduce them exactly; the HIP path
    (Gumbel-max on the device) is pinned against the oracle's logits instead."""
    d = {}
    g = torch.Generator().manual_seed(61)
    M, D, K = 512, 32, 64
    x = torch.randn(1, M, D, generator=g)
    E = torch.randn(K, D, generator=g) * 0.7
    d["x"], d["embed"] = x.numpy(), E.numpy()
    for j, temp in enumerate((0.5, 4.0)):
        for mode in ("eval", "train"):
            vqm = ref.vq.VectorQuantize(dim=D, codebook_size=K)
            vqm._codebook.embed.copy_(E)
            vqm._codebook.embed_avg.copy_(E)
            vqm.train(mode == "train")
            torch.manual_seed(1000 + j)
            q, ind, loss, perp = vqm(x.clone(), svq_temp=temp)
            key = f"t{j}_{mode}"
            d[f"{key}_temp"] = np.float32(temp)
            d[f"{key}_seed"] = np.int64(1000 + j)
            d[f"{key}_ind"] = ind.numpy()
            d[f"{key}_perplexity"] = np.float32(perp)
            if mode == "train":
                d[f"{key}_post_cluster_size"] = vqm._codebook.cluster_size.numpy().copy()
                d[f"{key}_post_embed"] = vqm._codebook.embed.numpy().copy()
    np.savez_compressed(os.path.join(OUT, "g6_svq.npz"), **d)


# --------------------------------------------------------------------------- G7
def gen_rocket():
    """ROCKET features (evaluation/rocket_functions.py:21-118).  numba is absent, so the
    file is loaded with `njit` as an identity decorator and `prange` as `range`: the same
    Python source, run by the interpreter in float64 (numba's fastmath may reassociate;
    the tests' tolerances cover it).  generate_kernels then draws from numpy's global RNG
    (under numba it would draw from numba's own stream), seeded below."""
    numba = types.ModuleType("numba")

    def njit(*a, **k):
        if len(a) == 1 and callable(a[0]) and not k:
            return a[0]
        return lambda f: f
    numba.njit = njit
    numba.prange = range
    sys.modules["numba"] = numba
    if not hasattr(np, "NINF"):  # numpy >= 2 dropped the alias the reference uses (:67)
        np.NINF = -np.inf
    rk = _load("ref_rocket", f"{REF}/evaluation/rocket_functions.py")
    d = {}
    for tag, (n, L, nk, seed) in {"a": (6, 128, 64, 7), "b": (3, 256, 40, 8)}.items():
        np.random.seed(seed)
        kern = rk.generate_kernels(L, nk)
        X = np.cumsum(np.random.randn(n, L), axis=1)
        X[0, :] = 0.0  # an all-zero series: every sum equals the bias
        feats = rk.apply_kernels(X, kern)
        w, lengths, biases, dil, pad = kern
        d[f"{tag}_X"], d[f"{tag}_weights"], d[f"{tag}_lengths"] = X, w, lengths
        d[f"{tag}_biases"], d[f"{tag}_dilations"], d[f"{tag}_paddings"] = biases, dil, pad
        d[f"{tag}_features"] = feats
    np.savez_compressed(os.path.join(OUT, "g7_rocket.npz"), **d)


# --------------------------------------------------------------------------- G8
FE_CONFIG = {"dim": 8, "dim_mults": [1, 2, 4, 8], "resnet_block_groups": 4, "dropout": 0.5}


def gen_fe(ref):
    """FidelityEnhancer eval forward (fidelity_enhancer.py:458-498, Unet1D :284-455) with
    configs/config.yaml:69-77 hyper-parameters.  Parameters come from param_init's per-key
    rule (seed 11), so only inputs and outputs are stored.  Case a: input_length 256 (the
    sampler's shape); case b: input_length 301 (the file's own __main__ length) with a
    256-long x_a, so the FE's interpolation and every ragged skip interpolation run."""
    fe_mod = _load("ref_fidelity_enhancer", f"{REF}/models/fidelity_enhancer.py")
    d = {}
    for tag, (B, C, Lx, Lin, seed) in {"a": (4, 6, 256, 256, 11), "b": (3, 6, 256, 301, 12)}.items():
        torch.manual_seed(seed)
        np.random.seed(seed)
        fe = fe_mod.FidelityEnhancer(Lin, C, {"fidelity_enhancer": dict(FE_CONFIG)})
        vals = fill_state_dict(fe.state_dict(), seed)
        fe.load_state_dict({k: torch.from_numpy(v) for k, v in vals.items()})
        fe.eval()
        g = torch.Generator().manual_seed(seed)
        x = torch.cumsum(0.1 * torch.randn(B, C, Lx, generator=g), -1)
        with torch.no_grad():
            y = fe(x)
        d[f"{tag}_x"], d[f"{tag}_y"] = x.numpy(), y.numpy()
        d[f"{tag}_meta"] = np.array([B, C, Lx, Lin, seed], dtype=np.int64)
        d[f"{tag}_keys"] = np.array(sorted(fe.state_dict().keys()))
    np.savez_compressed(os.path.join(OUT, "g8_fe.npz"), **d)


def _ref_fe(fe_mod, Lin, C, seed):
    """Reference FidelityEnhancer with dropout 0 (config.yaml's other FE settings) and
    param_init weights (seed), in training mode."""
    cfg = dict(FE_CONFIG)
    cfg["dropout"] = 0.0
    torch.manual_seed(seed)
    fe = fe_mod.FidelityEnhancer(Lin, C, {"fidelity_enhancer": cfg})
    vals = fill_state_dict(fe.state_dict(), seed)
    fe.load_state_dict({k: torch.from_numpy(v) for k, v in vals.items()})
    return fe.train()


def gen_fe_train(ref):
    """G11: Stage3 training (trainers/stage3.py:197-231) with dropout 0.
    Cases a / b: FidelityEnhancer forward + L1 loss + backward (fidelity_enhancer.py:458-498,
    stage3.py:206-209) at input_length 256 and 301 (ragged skips).  Case s3: the reference
    Stage3._fidelity_enhancer_loss_fn itself (stage3.py:193-210) -- decode LF / HF token
    indices with the reference MaskGIT over the G3-small stage1 (seed 3), FE, L1 -- loaded
    from the file with stubs for its plotting / evaluation imports; the stochastic-VQ
    encoding that produces the indices (svq_temp = tau) is pinned by G6."""
    fe_mod = _load("ref_fidelity_enhancer_t", f"{REF}/models/fidelity_enhancer.py")
    d = {}
    for tag, (B, C, Lx, Lin, seed) in {"a": (3, 6, 256, 256, 21), "b": (2, 6, 256, 301, 22)}.items():
        fe = _ref_fe(fe_mod, Lin, C, seed)
        g = torch.Generator().manual_seed(seed + 1)
        xp = torch.cumsum(0.1 * torch.randn(B, C, Lx, generator=g), -1)
        x = torch.cumsum(0.1 * torch.randn(B, C, Lin, generator=g), -1)
        xhat = fe(xp)
        loss = F.l1_loss(xhat, x)
        loss.backward()
        d[f"{tag}_xprime"], d[f"{tag}_x"] = xp.numpy(), x.numpy()
        d[f"{tag}_xhat"], d[f"{tag}_loss"] = xhat.detach().numpy(), np.array(float(loss))
        d[f"{tag}_meta"] = np.array([B, C, Lx, Lin, seed], dtype=np.int64)
        for k, prm in fe.named_parameters():
            if prm.grad is not None:
                d[f"{tag}_grad/{k}"] = prm.grad.numpy().copy()
    # ---- s3: the reference Stage3 loss function
    for name in ("timevqvae.evaluation", "timevqvae.trainers"):
        m = types.ModuleType(name)
        m.Metrics = m.MiniRocketTransform = m.Stage2 = object
        sys.modules[name] = m
    sys.modules["timevqvae.models"].FidelityEnhancer = fe_mod.FidelityEnhancer
    st3 = _load("ref_stage3", f"{REF}/trainers/stage3.py")
    T, Ks, hid, seed = 128, 64, 32, 3
    torch.manual_seed(seed)
    s1 = ref.stage1.Stage1(T, 6, _stage1_config(4, hid, Ks))
    vals = fill_state_dict(s1.state_dict(), seed)
    s1.load_state_dict({k: torch.from_numpy(v) for k, v in vals.items()}, strict=False)
    s1.eval()
    gx = torch.Generator().manual_seed(81)
    B = 4
    x = torch.cumsum(0.1 * torch.randn(B, 6, T, generator=gx), -1)
    with torch.no_grad():
        s1.encoder_l(x), s1.encoder_h(x)  # num_tokens / H' / W' buffers
    MG = ref.maskgit.MaskGIT
    mg = MG.__new__(MG)
    nn.Module.__init__(mg)
    for n in ("encoder_l", "decoder_l", "vq_model_l", "encoder_h", "decoder_h", "vq_model_h"):
        setattr(mg, n, getattr(s1, n))
    mg.H_prime_l, mg.W_prime_l = int(s1.encoder_l.H_prime), int(s1.encoder_l.W_prime)
    mg.H_prime_h, mg.W_prime_h = int(s1.encoder_h.H_prime), int(s1.encoder_h.W_prime)
    n_l, n_h = int(s1.encoder_l.num_tokens), int(s1.encoder_h.num_tokens)
    s_l = torch.randint(0, Ks, (B, n_l), generator=gx)
    s_h = torch.randint(0, Ks, (B, n_h), generator=gx)
    fe = _ref_fe(fe_mod, T, 6, 23)
    this = types.SimpleNamespace(maskgit=mg, fidelity_enhancer=fe)
    loss, (xprime, xhat) = st3.Stage3._fidelity_enhancer_loss_fn(this, x, s_l, s_h)
    loss.backward()
    d["s3_x"], d["s3_s_l"], d["s3_s_h"] = x.numpy(), s_l.numpy(), s_h.numpy()
    d["s3_xprime"], d["s3_xhat"] = xprime.numpy(), xhat.detach().numpy()
    d["s3_loss"] = np.array(float(loss))
    for k, prm in fe.named_parameters():
        if prm.grad is not None:
            d[f"s3_grad/{k}"] = prm.grad.numpy().copy()
    np.savez_compressed(os.path.join(OUT, "g11_fe_train.npz"), **d)
    print("g11", {k: float(d[k]) for k in ("a_loss", "b_loss", "s3_loss")})


# --------------------------------------------------------------------------- G9
def install_x_transformers_stub():
    """x-transformers (pyproject.toml:21, ^1.31.6) is absent from the image and has no
    source on disk, so bidirectional_transformer.py:8-9 cannot import it.  This stub
    registers a module `x_transformers` whose ContinuousTransformerWrapper / Encoder
    are the T1 restatement (x-transformers 1.3x behaviour, the same arithmetic as
    oracle/tvq_oracle.py:xf_blocks) with the x-transformers module tree, so the
    reference file itself runs: Upscale, embeddings, class conditioning, pred_head,
    tied logits and the MaskGIT loss composition are then the reference's own code.
    Only T1's arithmetic stays parity-unpinned."""
    import random
    import torch.nn.functional as F

    xt = types.ModuleType("x_transformers")

    class RMSNorm(nn.Module):  # F.normalize(x) * sqrt(dim) * g
        def __init__(self, dim):
            super().__init__()
            self.scale = dim ** 0.5
            self.g = nn.Parameter(torch.ones(dim))

        def forward(self, x):
            return F.normalize(x, dim=-1) * self.scale * self.g

    class LayerNorm(nn.Module):  # gamma-only LayerNorm (beta is a zero buffer)
        def __init__(self, dim):
            super().__init__()
            self.gamma = nn.Parameter(torch.ones(dim))
            self.register_buffer("beta", torch.zeros(dim), persistent=False)

        def forward(self, x):
            return F.layer_norm(x, x.shape[-1:], self.gamma, self.beta)

    class Attention(nn.Module):
        def __init__(self, dim, heads, dim_head, dropout):
            super().__init__()
            self.heads, self.dim_head = heads, dim_head
            inner = heads * dim_head
            self.to_q = nn.Linear(dim, inner, bias=False)
            self.to_k = nn.Linear(dim, inner, bias=False)
            self.to_v = nn.Linear(dim, inner, bias=False)
            self.to_out = nn.Linear(inner, dim, bias=False)
            self.dropout = nn.Dropout(dropout)

        def forward(self, x):
            B, S, _ = x.shape
            sh = lambda t: t.view(B, S, self.heads, self.dim_head).transpose(1, 2)
            q, k, v = sh(self.to_q(x)), sh(self.to_k(x)), sh(self.to_v(x))
            att = torch.softmax(q @ k.transpose(-1, -2) * self.dim_head ** -0.5, dim=-1)
            o = (self.dropout(att) @ v).transpose(1, 2).reshape(B, S, -1)
            return self.to_out(o)

    class FeedForward(nn.Module):
        def __init__(self, dim, mult, dropout):
            super().__init__()
            inner = int(dim * mult)
            self.ff = nn.Sequential(nn.Sequential(nn.Linear(dim, inner), nn.GELU()),
                                    nn.Dropout(dropout), nn.Linear(inner, dim))

        def forward(self, x):
            return self.ff(x)

    class Residual(nn.Module):
        def forward(self, x, residual):
            return x + residual

    class Encoder(nn.Module):
        def __init__(self, dim, depth, heads=8, pre_norm=True, use_rmsnorm=False,
                     layer_dropout=0.0, **kw):
            super().__init__()
            assert pre_norm
            self.dim = dim
            norm = (lambda: RMSNorm(dim)) if use_rmsnorm else (lambda: LayerNorm(dim))
            dim_head = kw.get("attn_dim_head", 64)
            self.layers = nn.ModuleList()
            for t in ("a", "f") * depth:
                block = (Attention(dim, heads, dim_head, kw.get("attn_dropout", 0.0)) if t == "a"
                         else FeedForward(dim, kw.get("ff_mult", 4), kw.get("ff_dropout", 0.0)))
                self.layers.append(nn.ModuleList([nn.ModuleList([norm(), None, None]), block,
                                                  Residual()]))
            self.layer_dropout = layer_dropout
            self.final_norm = norm()

        def forward(self, x):
            for norms, block, residual_fn in self.layers:
                if self.training and self.layer_dropout > 0.0 and random.random() < self.layer_dropout:
                    continue
                x = residual_fn(block(norms[0](x)), x)
            return self.final_norm(x)

    class ContinuousTransformerWrapper(nn.Module):
        def __init__(self, *, max_seq_len, attn_layers, dim_in=None, dim_out=None,
                     use_abs_pos_emb=True, post_emb_norm=False, emb_dropout=0.0, **kw):
            super().__init__()
            assert not use_abs_pos_emb
            dim = attn_layers.dim
            self.max_seq_len = max_seq_len
            self.post_emb_norm = LayerNorm(dim) if post_emb_norm else nn.Identity()
            self.emb_dropout = nn.Dropout(emb_dropout)
            self.project_in = nn.Linear(dim_in, dim, bias=False) if dim_in is not None else nn.Identity()
            self.attn_layers = attn_layers
            self.project_out = nn.Linear(dim, dim_out, bias=False) if dim_out is not None else nn.Identity()

        def forward(self, x):
            x = self.post_emb_norm(self.project_in(x))
            x = self.attn_layers(self.emb_dropout(x))
            return self.project_out(x)

    xt.ContinuousTransformerWrapper = ContinuousTransformerWrapper
    xt.Encoder = Encoder
    sys.modules["x_transformers"] = xt
    return xt


def load_reference_stage2(ref):
    """bidirectional_transformer.py (with the x_transformers stub) + maskgit.py re-loaded
    against it."""
    install_x_transformers_stub()
    bt = _load("ref_bidirectional_transformer", f"{REF}/models/bidirectional_transformer.py")
    sys.modules["timevqvae.models"].BidirectionalTransformer = bt.BidirectionalTransformer
    maskgit = _load("ref_maskgit_bt", f"{REF}/models/maskgit.py")
    return bt, maskgit


PRIOR_L = {"hidden_dim": 128, "n_layers": 4, "heads": 2, "ff_mult": 1, "use_rmsnorm": True}
PRIOR_H = {"hidden_dim": 32, "n_layers": 1, "heads": 1, "ff_mult": 1, "use_rmsnorm": True}


def gout(shape, seed):
    """Upstream gradient for the G9 backward checks (numpy, so tests rebuild it)."""
    return np.random.default_rng(seed + 200).standard_normal(shape).astype(np.float32)


class _Recorder:
    """Records every torch.rand / np.random.uniform draw the reference makes (in call
    order), so the HIP path can be fed the same draws."""

    def __init__(self):
        self.torch_rand, self.np_uniform = [], []

    def __enter__(self):
        self._tr, self._nu = torch.rand, np.random.uniform

        def tr(*a, **k):
            t = self._tr(*a, **k)
            self.torch_rand.append(t.detach().clone())
            return t

        def nu(*a, **k):
            v = self._nu(*a, **k)
            self.np_uniform.append(np.array(v, dtype=np.float64).copy())
            return v
        torch.rand, np.random.uniform = tr, nu
        return self

    def __exit__(self, *exc):
        torch.rand, np.random.uniform = self._tr, self._nu


def gen_stage2(ref):
    """G9: the reference BidirectionalTransformer (bidirectional_transformer.py:34-251)
    and MaskGIT forward / CFG (maskgit.py:136-192) run from the reference files, with
    x-transformers replaced by the restated stub (install_x_transformers_stub).  Params
    come from param_init (seeded per key); every random draw is recorded and stored."""
    bt, maskgit = load_reference_stage2(ref)
    d = {}
    K, B, emb = 512, 4, 128
    # ---- (1) transformers alone at the config-B architecture (K=512, hid 128)
    for kind, pm, seed in (("lf", PRIOR_L, 41), ("hf", PRIOR_H, 42)):
        torch.manual_seed(seed)
        m = bt.BidirectionalTransformer(kind, 24 if kind == "lf" else 96, {"lf": K, "hf": K}, emb,
                                        p_unconditional=0.2, n_classes=5, model_dropout=0.0,
                                        emb_dropout=0.0, num_tokens_l=24, **pm)
        vals = fill_state_dict(m.state_dict(), seed)
        m.load_state_dict({k: torch.from_numpy(v) for k, v in vals.items()}, strict=True)
        g = torch.Generator().manual_seed(seed + 100)
        s_l = torch.randint(0, K + 1, (B, 24), generator=g)
        s_h = torch.randint(0, K + 1, (B, 96), generator=g)
        s_l[:, :5] = K  # some mask tokens
        s_h[:, ::3] = K
        y = torch.randint(0, 5, (B, 1), generator=g)
        args = (s_l,) if kind == "lf" else (s_l, s_h)
        p = f"{kind}_"
        d[p + "s_l"], d[p + "s_h"], d[p + "y"] = s_l.numpy(), s_h.numpy(), y.numpy()
        d[p + "keys"] = np.array(sorted(m.state_dict().keys()))
        m.eval()
        with torch.no_grad():
            d[p + "eval_cond"] = m(*args, class_condition=y).numpy()
            d[p + "eval_uncond"] = m(*args, class_condition=None).numpy()
        m.train()  # train-mode BN (Upscale), class-drop draws recorded
        with _Recorder() as rec:
            logits = m(*args, class_condition=y)
        d[p + "train_cls_rand"] = rec.torch_rand[0].numpy()
        d[p + "train_cond"] = logits.detach().numpy()
        gl = torch.from_numpy(gout(logits.shape, seed))  # regenerated by the tests
        (logits * gl).sum().backward()
        for k, prm in m.named_parameters():
            if prm.grad is not None:
                d[p + "grad/" + k] = prm.grad.numpy().copy()
        d.update({p + "post/" + k: v.numpy().copy() for k, v in m.state_dict().items()
                  if k.endswith(("running_mean", "running_var"))})

    # ---- (2) MaskGIT.forward loss (maskgit.py:155-192) over a stage1 (T=128, K=64, hid 32)
    T, Ks, hid = 128, 64, 32
    seed = 3  # the G3-small stage1 weights
    cfg = _stage1_config(4, hid, Ks)
    torch.manual_seed(seed)
    s1 = ref.stage1.Stage1(T, 6, cfg)
    vals = fill_state_dict(s1.state_dict(), seed)
    s1.load_state_dict({k: torch.from_numpy(v) for k, v in vals.items()}, strict=False)
    gx = torch.Generator().manual_seed(77)
    Bm = 8
    x = torch.cumsum(0.1 * torch.randn(Bm, 6, T, generator=gx), -1)
    x = 2 * (x - x.amin(0, keepdim=True)) / (x.amax(0, keepdim=True) - x.amin(0, keepdim=True) + 1e-8) - 1
    y = torch.randint(0, 5, (Bm, 1), generator=gx)
    s1.eval()
    with torch.no_grad():
        s1.encoder_l(x), s1.encoder_h(x)  # sets num_tokens / H' / W' buffers (vq_vae.py:183-187)
    MG = maskgit.MaskGIT
    mg = MG.__new__(MG)
    nn.Module.__init__(mg)
    mg.choice_temperature_l, mg.choice_temperature_h = 10, 4
    mg.T = {"lf": 10, "hf": 1}
    mg.n_classes = 5
    mg.cfg_scale = 1.0
    mg.mask_token_ids = {"lf": Ks, "hf": Ks}
    mg.gamma = mg.gamma_func("cosine")
    mg.stage1 = s1
    for n in ("encoder_l", "decoder_l", "vq_model_l", "encoder_h", "decoder_h", "vq_model_h"):
        setattr(mg, n, getattr(s1, n))
    mg.num_tokens_l, mg.num_tokens_h = int(s1.encoder_l.num_tokens), int(s1.encoder_h.num_tokens)
    prior = dict(p_unconditional=0.2, model_dropout=0.0, emb_dropout=0.0)
    torch.manual_seed(50)
    mg.transformer_l = bt.BidirectionalTransformer("lf", mg.num_tokens_l, {"lf": Ks, "hf": Ks}, hid,
                                                   n_classes=5, **PRIOR_L, **prior)
    mg.transformer_h = bt.BidirectionalTransformer("hf", mg.num_tokens_h, {"lf": Ks, "hf": Ks}, hid,
                                                   n_classes=5, num_tokens_l=mg.num_tokens_l,
                                                   **PRIOR_H, **prior)
    for name in ("transformer_l", "transformer_h"):
        tm = getattr(mg, name)
        vals = fill_state_dict(tm.state_dict(), 50)
        tm.load_state_dict({k: torch.from_numpy(v) for k, v in vals.items()}, strict=True)
    for p_ in s1.parameters():
        p_.requires_grad_(False)
    mg.train()
    np.random.seed(31)
    torch.manual_seed(32)
    with _Recorder() as rec:
        loss, (loss_l, loss_h) = mg(x, y)
    # draw order (maskgit.py:167-178, bidirectional_transformer.py:140-143):
    # np ratio_l, torch rand_l, np ratio_h, torch rand_h, cls rand (LF), cls rand (HF)
    assert len(rec.np_uniform) == 2 and len(rec.torch_rand) == 4, (len(rec.np_uniform), len(rec.torch_rand))
    d["mg_x"], d["mg_y"] = x.numpy(), y.numpy()
    d["mg_ratio_l"], d["mg_ratio_h"] = rec.np_uniform
    d["mg_rand_l"], d["mg_rand_h"] = rec.torch_rand[0].numpy(), rec.torch_rand[1].numpy()
    d["mg_cls_rand_l"], d["mg_cls_rand_h"] = rec.torch_rand[2].numpy(), rec.torch_rand[3].numpy()
    d["mg_loss"], d["mg_loss_l"], d["mg_loss_h"] = (np.array(float(v)) for v in (loss, loss_l, loss_h))
    loss.backward()
    for name in ("transformer_l", "transformer_h"):
        for k, prm in getattr(mg, name).named_parameters():
            if prm.grad is not None:
                d[f"mg_grad/{name}.{k}"] = prm.grad.numpy().copy()
        for k, v in getattr(mg, name).state_dict().items():
            if k.endswith(("running_mean", "running_var")):  # Upscale BN after the forward
                d[f"mg_post/{name}.{k}"] = v.numpy().copy()
    with torch.no_grad():
        _, s_l = mg.encode_to_z_q(x, mg.encoder_l, mg.vq_model_l)
        _, s_h = mg.encode_to_z_q(x, mg.encoder_h, mg.vq_model_h)
    d["mg_s_l"], d["mg_s_h"] = s_l.numpy().astype(np.int64), s_h.numpy().astype(np.int64)

    # ---- (3) masked_prediction with classifier-free guidance (maskgit.py:136-153), eval
    mg.eval()
    mg.cfg_scale = 2.0
    gs = torch.Generator().manual_seed(78)
    s_l_M = torch.randint(0, Ks + 1, s_l.shape, generator=gs)
    s_h_M = torch.randint(0, Ks + 1, s_h.shape, generator=gs)
    with torch.no_grad():
        d["cfg_s_l_M"], d["cfg_s_h_M"] = s_l_M.numpy(), s_h_M.numpy()
        d["cfg_logits_l"] = mg.masked_prediction(mg.transformer_l, y, s_l_M).numpy()
        d["cfg_logits_h"] = mg.masked_prediction(mg.transformer_h, y, s_l_M, s_h_M).numpy()
        d["cfg_logits_h_uncond"] = mg.masked_prediction(mg.transformer_h, None, s_l_M, s_h_M).numpy()
    np.savez_compressed(os.path.join(OUT, "g9_stage2.npz"), **d)


def gen_fid(ref):
    """G10: calculate_fid (evaluation/eval_utils.py:56-81), loaded by file path (its
    FCNBaseline import is stubbed: the function never uses it).  Case a: float64 Gaussian
    features, D=32; b: ROCKET-like float64 features (ppv in [0,1] | max), D=160; c: float32
    FCN-like features, D=128 (the reference takes the mean in float32, the cov in float64)."""
    sys.modules["timevqvae.models"].FCNBaseline = object
    eu = _load("ref_eval_utils", f"{REF}/evaluation/eval_utils.py")
    rng = np.random.default_rng(10)
    d = {}
    A = rng.standard_normal((32, 32)) / 6
    Bm = rng.standard_normal((32, 32)) / 5
    cases = {
        "a": (rng.standard_normal((600, 32)) @ A, 0.3 + rng.standard_normal((500, 32)) @ Bm),
        "b": (np.concatenate([rng.uniform(0, 1, (700, 80)), rng.normal(1.0, 2.0, (700, 80))], 1),
              np.concatenate([rng.uniform(0.1, 1, (600, 80)), rng.normal(1.2, 1.8, (600, 80))], 1)),
        "c": (rng.standard_normal((700, 128)).astype(np.float32),
              (0.1 + 1.1 * rng.standard_normal((650, 128))).astype(np.float32)),
    }
    for k, (z1, z2) in cases.items():
        d[f"{k}_z1"], d[f"{k}_z2"] = z1, z2
        d[f"{k}_fid"] = np.float64(eu.calculate_fid(z1, z2))
        for i, z in ((1, z1), (2, z2)):
            d[f"{k}_mu{i}"] = np.asarray(z.mean(axis=0), np.float64)
            d[f"{k}_sigma{i}"] = np.cov(z, rowvar=False)
        print("fid", k, d[f"{k}_fid"])
    np.savez_compressed(os.path.join(OUT, "g10_fid.npz"), **d)


def main():
    torch.set_num_threads(8)
    if sys.argv[1:] == ["rocket"]:  # regenerate only G7
        gen_rocket()
        return
    ref = load_reference()
    if sys.argv[1:] == ["svq"]:  # regenerate only G6
        gen_svq(ref)
        return
    if sys.argv[1:] == ["fe"]:  # regenerate only G8
        gen_fe(ref)
        return
    if sys.argv[1:] == ["stage2"]:  # regenerate only G9
        gen_stage2(ref)
        return
    if sys.argv[1:] == ["fetrain"]:  # regenerate only G11
        gen_fe_train(ref)
        return
    if sys.argv[1:] == ["fid"]:  # regenerate only G10
        gen_fid(ref)
        return
    if sys.argv[1:] == ["cfgA"]:  # regenerate only G3 at BASELINE configs[0]
        gen_stage1(ref, "cfgA", B=4, C=6, T=128, K=256, init_dim=4, hid_dim=128, seed=7)
        return
    gen_vq(ref)
    gen_stft(ref)
    gen_stage1(ref, "small", B=4, C=6, T=128, K=64, init_dim=4, hid_dim=32, seed=3)
    gen_stage1(ref, "cfgB", B=2, C=6, T=256, K=512, init_dim=4, hid_dim=128, seed=5)
    gen_stage1(ref, "cfgA", B=4, C=6, T=128, K=256, init_dim=4, hid_dim=128, seed=7)
    gen_maskgit(ref)
    gen_svq(ref)
    gen_rocket()
    gen_fe(ref)
    gen_fid(ref)
    gen_fe_train(ref)
    for f in sorted(os.listdir(OUT)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(OUT, f)))


if __name__ == "__main__":
    main()
