"""The oracle's Stage1 restatement (tvq_oracle.stage1_forward) pinned to the reference's own
step (G3, tests/golden/make_golden.py ran trainers/stage1.py on these weights): losses, code
indices, every parameter gradient (CPU autograd through the restatement) and every buffer
update (BN running statistics, VQ EMA).  This is what lets tests/test_fullsize_parity.py use
the oracle as the checker at B=256, a batch the goldens do not cover.  CPU only.

Tolerances: the reference's and the restatement's arithmetic are both torch CPU fp32, so
losses within 1e-5 relative, gradients per tensor within 1e-5 max|g_ref| + 1e-8 (a conv bias
feeding a BatchNorm is scaled by its weight's gradient: its true value is 0), indices equal.
"""
import numpy as np
import pytest
import torch

from oracle import tvq_oracle as O
from test_stage1 import TAGS, build


@pytest.mark.parametrize("tag", TAGS)
def test_oracle_stage1_step_matches_reference(tag):
    m, g = build(tag)
    Bg, Cg, Tg, Kg, init_dim, hid_dim = [int(v) for v in g["cfg"]]
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    params = {k: sd[k].clone().requires_grad_(True) for k, _ in m.named_parameters()}
    sdo = dict(sd)
    sdo.update(params)
    ctx = O.Ctx(True)
    spec = O.Stage1Spec(Tg, Cg, init_dim, hid_dim)
    out = O.stage1_forward(ctx, sdo, spec, torch.from_numpy(g["x"]))
    out["loss"].backward()
    for k, gk in (("loss", "train_loss"), ("recons_lf", "train_recons_lf"),
                  ("recons_hf", "train_recons_hf"), ("commit_lf", "train_commit_lf"),
                  ("commit_hf", "train_commit_hf"), ("perp_lf", "train_perp_lf"),
                  ("perp_hf", "train_perp_hf")):
        v, r = float(out[k].detach()), float(g[gk])
        assert abs(v - r) <= 1e-5 * abs(r) + 1e-8, (k, v, r)
    assert np.array_equal(out["s_l"].numpy().reshape(-1), g["train_vq_model_l_ind"].reshape(-1))
    assert np.array_equal(out["s_h"].numpy().reshape(-1), g["train_vq_model_h_ind"].reshape(-1))
    bad = []
    for k, p in params.items():
        r = g["grad/" + k]
        d = p.grad.numpy()
        scale = np.abs(r).max()
        wk = "grad/" + k[: -len("bias")] + "weight"
        if k.endswith(".bias") and wk in g and g[wk].ndim >= 3:
            scale = max(scale, np.abs(g[wk]).max())
        if np.abs(d - r).max() > 1e-5 * scale + 1e-8:
            bad.append((k, float(np.abs(d - r).max()), float(scale)))
    assert not bad, bad[:6]
    badb = []
    for k, v in ctx.updates.items():
        r = g["post/" + k]
        v = v.detach().numpy()
        if v.dtype.kind == "f":
            err = np.abs(v - r).max() / (np.abs(r).max() + 1e-12)
            if err > 1e-5:
                badb.append((k, float(err)))
        elif not np.array_equal(v, r):
            badb.append((k, "int"))
    assert not badb, badb[:6]
    updated = {k for k in g.files if k.startswith("post/") and k.endswith(
        ("running_mean", "running_var", "num_batches_tracked", "cluster_size", "embed_avg", "embed"))}
    assert set("post/" + k for k in ctx.updates) == updated
