"""Stage1 end to end vs the reference goldens (G3): eval reconstruction, train-mode
losses, code indices, every parameter gradient and the buffer updates (BN running
stats, VQ EMA).  Dropout off: the goldens were made with p = 0.

Tolerances: reconstructions/losses rel <= 1e-4 (north_star); gradients
|g - g_ref| <= 1e-4 * max|g_ref| + 1e-6 per tensor (conv biases feeding a BatchNorm
have a mathematically zero gradient, pure rounding noise ~1e-9, hence the atol).
"""
import numpy as np
import pytest
import torch

from conftest import golden
from param_init import fill_state_dict

TAGS = ["small", "cfgB", "cfgA"]  # cfgA: BASELINE configs[0] (T=128, K=256, hid 128)


def make_config(K, init_dim, hid_dim):
    return {
        "VQ-VAE": {"n_fft": 4, "codebook_sizes": {"lf": K, "hf": K}},
        "encoder": {"init_dim": init_dim, "hid_dim": hid_dim, "n_resnet_blocks": 2,
                    "downsampled_width": {"lf": 8, "hf": 32}},
        "decoder": {"n_resnet_blocks": 2},
        "exp_params": {"lr": 1e-3, "linear_warmup_rate": 0.1},
        "trainer_params": {"max_steps": {"stage1": 1000, "stage2": 1000}},
    }


def build(tag, device=None):
    from timevqvae.trainers import Stage1
    g = golden(f"g3_stage1_{tag}.npz")
    B, C, T, K, init_dim, hid_dim = [int(v) for v in g["cfg"]]
    m = Stage1(T, C, make_config(K, init_dim, hid_dim))
    vals = fill_state_dict(m.state_dict(), int(g["seed"]))
    m.load_state_dict({k: torch.from_numpy(v) for k, v in vals.items()}, strict=False)
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    if device is not None:
        m = m.to(device)
    return m, g


@pytest.mark.parametrize("tag", TAGS)
def test_stage1_module_tree_matches_reference(tag):
    """state_dict keys and shapes equal the reference's (checkpoint compatibility)."""
    m, g = build(tag)
    sd = m.state_dict()
    ref_params = {k[5:]: g[k].shape for k in g if k.startswith("grad/")}
    ref_bufs = {k[5:]: g[k].shape for k in g if k.startswith("post/")}
    mine_params = {k: tuple(p.shape) for k, p in m.named_parameters()}
    assert mine_params == {k: tuple(v) for k, v in ref_params.items()}
    for k, shp in ref_bufs.items():
        assert k in sd, k
        assert tuple(sd[k].shape) == tuple(shp), k


def _index_ok(got, want, z_tokens, embed):
    from oracle import vq_ref
    bad = np.nonzero(got.reshape(-1) != want.reshape(-1))[0]
    if len(bad) == 0:
        return True
    _, _, gap = vq_ref.assign(z_tokens, embed)
    tol = 1e-5 * ((z_tokens.astype(np.float64) ** 2).sum(1) + (embed.astype(np.float64) ** 2).sum(1).max())
    return all(gap[i] <= tol[i] for i in bad)


@pytest.mark.gpu
@pytest.mark.parametrize("tag", TAGS)
def test_stage1_eval_reconstruction(tag, cuda):
    m, g = build(tag, cuda)
    m.eval()
    x = torch.from_numpy(g["x"]).to(cuda)
    with torch.no_grad():
        xr = m((x, None), 0, return_x_rec=True).cpu().numpy()
        z_l = m.encoder_l(x).cpu().numpy()
        z_h = m.encoder_h(x).cpu().numpy()
    ref = g["eval_x_rec"]
    assert np.linalg.norm(xr - ref) / np.linalg.norm(ref) < 1e-4
    for z, k in ((z_l, "eval_z_l"), (z_h, "eval_z_h")):
        assert np.linalg.norm(z - g[k]) / np.linalg.norm(g[k]) < 1e-5, k


@pytest.mark.gpu
@pytest.mark.parametrize("tag,flat", [("small", False), ("cfgB", False), ("cfgB", True),
                                      ("cfgA", True)])
def test_stage1_train_step_grads(tag, flat, cuda):
    """flat=True: FusedAdamW owns the gradients (kernels accumulate into the flat buffer)."""
    m, g = build(tag, cuda)
    if flat:
        from timevqvae.hip.optim import FusedAdamW
        opt = FusedAdamW(m.parameters(), lr=1e-3)
        opt.zero_grad()
    embeds = {n: getattr(m, n)._codebook.embed.detach().cpu().numpy().copy()
              for n in ("vq_model_l", "vq_model_h")}
    m.train()
    cap = {}
    for n in ("vq_model_l", "vq_model_h"):
        getattr(m, n).register_forward_hook(
            lambda mod, inp, o, n=n: cap.__setitem__(n, o[1].detach().cpu().numpy()))
    x = torch.from_numpy(g["x"]).to(cuda)
    out = m.training_step((x, None), 0)
    out["loss"].sum().backward()
    torch.cuda.synchronize()
    for k, gk in (("loss", "train_loss"), ("recons_loss.LF.time", "train_recons_lf"),
                  ("recons_loss.HF.time", "train_recons_hf"), ("commit_loss.LF", "train_commit_lf"),
                  ("commit_loss.HF", "train_commit_hf"), ("perplexity.LF", "train_perp_lf"),
                  ("perplexity.HF", "train_perp_hf")):
        v = float(out[k].detach().sum())
        assert abs(v - float(g[gk])) <= 1e-4 * abs(float(g[gk])) + 1e-7, (k, v, float(g[gk]))
    # code indices: exact unless the reference z sits on an fp32 near-tie
    for n, zk, ik in (("vq_model_l", "train_encoder_l", "train_vq_model_l_ind"),
                      ("vq_model_h", "train_encoder_h", "train_vq_model_h_ind")):
        z = g[zk]
        zt = z.transpose(0, 2, 3, 1).reshape(-1, z.shape[1])
        assert _index_ok(cap[n], g[ik], zt, embeds[n]), n
    bad = []
    for k, p in m.named_parameters():
        r = g["grad/" + k]
        d = p.grad.detach().cpu().numpy()
        scale = np.abs(r).max()
        wk = "grad/" + k[: -len("bias")] + "weight"
        if k.endswith(".bias") and wk in g and g[wk].ndim >= 3:
            # conv bias: when a BatchNorm follows, its true gradient is 0 (pure noise)
            scale = max(scale, np.abs(g[wk]).max())
        if np.abs(d - r).max() > 1e-4 * scale + 1e-6:
            bad.append((k, float(np.abs(d - r).max()), float(np.abs(r).max())))
    assert not bad, bad[:6]
    sd = m.state_dict()
    badb = []
    for k in g:
        if not k.startswith("post/"):
            continue
        kk = k[5:]
        v = sd[kk].detach().cpu().numpy()
        r = g[k]
        if v.dtype.kind == "f":
            if kk.endswith("embed"):
                err = (np.abs(v - r) / np.linalg.norm(r, axis=-1, keepdims=True)).max()
            else:
                err = np.abs(v - r).max() / (np.abs(r).max() + 1e-12)
            if err > 1e-4:
                badb.append((kk, float(err)))
        else:
            if not np.array_equal(v, r):
                badb.append((kk, "int mismatch"))
    assert not badb, badb[:6]
