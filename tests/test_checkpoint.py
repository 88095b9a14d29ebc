"""Checkpoint compatibility: reference Lightning checkpoints load into
the HIP modules.

* stage1: a Lightning-shaped `stage1.ckpt` whose keys are the REFERENCE's own (taken from
  the G3 golden, which the reference Stage1 produced) loads strictly, and on the GPU
  reproduces the reference's eval reconstruction from it.
* stage2: save -> load round trip through `Stage2.load_from_checkpoint` as
  generation/sampler.py:76-90 calls it, with the x-transformers norm spellings of other
  releases (`gamma` for RMSNorm, `weight`/`bias` LayerNorm, zero Linear biases) adapted.
  The x-transformers layout itself is parity unpinned.
"""
import copy

import numpy as np
import pytest
import torch

from conftest import golden
from param_init import value_for
from test_stage1 import make_config


def _reference_stage1_ckpt(tag, path):
    """A Lightning checkpoint with the reference Stage1's key set and G3's weights."""
    g = golden(f"g3_stage1_{tag}.npz")
    seed = int(g["seed"])
    sd = {}
    for k in g.files:
        if k.startswith("grad/"):
            key = k[5:]
            sd[key] = torch.from_numpy(value_for(key, g[k].shape, seed))
        elif k.startswith("post/"):
            key = k[5:]
            v = g[k]
            sd[key] = (torch.from_numpy(value_for(key, v.shape, seed))
                       if v.dtype.kind == "f" else torch.from_numpy(np.array(v)))
    ckpt = {"epoch": 3, "global_step": 1200, "pytorch-lightning_version": "2.2.1",
            "state_dict": sd, "loops": {}, "callbacks": {},
            "optimizer_states": [{"state": {}, "param_groups": [{"lr": 1e-3, "params": [0]}]}],
            "lr_schedulers": [{"last_epoch": 1200}]}
    torch.save(ckpt, path)
    B, C, T, K, init_dim, hid_dim = [int(v) for v in g["cfg"]]
    return sd, g, (T, C, make_config(K, init_dim, hid_dim))


@pytest.mark.parametrize("tag", ["small", "cfgB"])
def test_stage1_loads_reference_keyed_checkpoint(tag, tmp_path):
    from timevqvae.trainers import Stage1
    path = tmp_path / "stage1.ckpt"
    sd, _, (T, C, cfg) = _reference_stage1_ckpt(tag, path)
    m = Stage1.load_from_checkpoint(str(path), input_length=T, in_channels=C, config=cfg,
                                    map_location="cpu")
    mine = m.state_dict()
    assert set(mine) == set(sd)
    for k, v in sd.items():
        assert torch.equal(mine[k], v.to(mine[k].dtype)), k


def test_checkpoint_refuses_non_tensor_payload(tmp_path):
    """Files are read with weights_only=True: a pickled object is refused, never run."""
    from timevqvae.utils.checkpoint import read_state_dict

    import argparse
    path = tmp_path / "evil.ckpt"
    torch.save({"state_dict": {}, "obj": argparse.Namespace(a=1)}, path)
    with pytest.raises(Exception):
        read_state_dict(str(path))


def _stage2_cfg():
    import bench
    cfg = copy.deepcopy(bench.config(False))
    cfg["VQ-VAE"]["codebook_sizes"] = {"lf": 64, "hf": 64}
    cfg["encoder"]["hid_dim"] = 32
    return cfg


def _randomize(m, seed):
    gen = torch.Generator().manual_seed(seed)
    sd = {}
    for k, v in m.state_dict().items():
        sd[k] = (torch.randn(v.shape, generator=gen) * 0.1 + (1.0 if k.endswith(("g", "gamma"))
                                                              else 0.0)
                 if v.is_floating_point() and "running_var" not in k else v)
    m.load_state_dict(sd)


def _xt_variant(sd):
    """Re-spell the transformer keys as another x-transformers release would."""
    out = {}
    for k, v in sd.items():
        if k.endswith(".0.0.g") or k.endswith("final_norm.g"):
            out[k[:-1] + "gamma"] = v
        elif k.endswith("post_emb_norm.gamma"):
            out[k[:-5] + "weight"] = v
            out[k[:-5] + "bias"] = torch.zeros_like(v)
        else:
            out[k] = v
        if k.endswith("blocks.project_in.weight"):
            out[k[:-6] + "bias"] = torch.zeros(v.shape[0])
    return out


def _build_stage2(tmp_path, cfg):
    from timevqvae.trainers import Stage1, Stage2
    s1 = Stage1(64, 6, cfg)
    _randomize(s1, 1)
    p1 = tmp_path / "stage1.ckpt"
    s1.save_checkpoint(str(p1))
    s2 = Stage2(str(p1), None, 64, 6, 5, config=cfg)
    _randomize(s2.maskgit.transformer_l, 2)
    _randomize(s2.maskgit.transformer_h, 3)
    return s2, p1


def test_stage2_checkpoint_roundtrip_with_xtransformers_variants(tmp_path):
    from timevqvae.trainers import Stage2
    cfg = _stage2_cfg()
    s2, p1 = _build_stage2(tmp_path, cfg)
    sd = s2.state_dict()
    p2 = tmp_path / "stage2.ckpt"
    torch.save({"epoch": 1, "state_dict": _xt_variant(sd)}, p2)
    kw = dict(stage1_ckpt_fname=str(p1), fcn_ckpt_fname=None, input_length=64, in_channels=6,
              n_classes=5, X_train=None, X_test=None, config=cfg, device="cpu",
              feature_extractor_type="rocket")
    m = Stage2.load_from_checkpoint(str(p2), map_location="cpu", **kw)
    got = m.state_dict()
    assert set(got) == set(sd)
    for k in sd:
        assert torch.equal(got[k], sd[k]), k
    # the stage1 weights inside stage2.ckpt suffice (no stage1 file)
    kw["stage1_ckpt_fname"] = None
    m2 = Stage2.load_from_checkpoint(str(p2), **kw)
    assert all(torch.equal(m2.state_dict()[k], sd[k]) for k in sd)


def test_stage2_checkpoint_rejects_nonidentity_extra_params(tmp_path):
    from timevqvae.trainers import Stage2
    cfg = _stage2_cfg()
    s2, p1 = _build_stage2(tmp_path, cfg)
    bad = _xt_variant(s2.state_dict())
    k = next(k for k in bad if k.endswith("project_in.bias"))
    bad[k] = torch.ones_like(bad[k])
    p2 = tmp_path / "stage2.ckpt"
    torch.save({"state_dict": bad}, p2)
    with pytest.raises(ValueError, match="project_in.bias"):
        Stage2.load_from_checkpoint(str(p2), stage1_ckpt_fname=str(p1), input_length=64,
                                    in_channels=6, n_classes=5, config=cfg)


@pytest.mark.gpu
def test_stage1_reference_checkpoint_reproduces_reference_reconstruction(tmp_path, cuda):
    """The loaded reference-keyed checkpoint reproduces the reference's eval output (G3)."""
    from timevqvae.trainers import Stage1
    path = tmp_path / "stage1.ckpt"
    _, g, (T, C, cfg) = _reference_stage1_ckpt("cfgB", path)
    m = Stage1.load_from_checkpoint(str(path), input_length=T, in_channels=C, config=cfg)
    m = m.to(cuda).eval()
    x = torch.from_numpy(g["x"]).to(cuda)
    with torch.no_grad():
        xr = m((x, None), 0, return_x_rec=True).cpu().numpy()
    ref = g["eval_x_rec"]
    assert np.linalg.norm(xr - ref) / np.linalg.norm(ref) < 1e-4


@pytest.mark.gpu
def test_stage2_loaded_checkpoint_same_logits(tmp_path, cuda):
    """A reloaded stage2 checkpoint (variant key spellings) gives identical logits."""
    from timevqvae.trainers import Stage2
    cfg = _stage2_cfg()
    s2, p1 = _build_stage2(tmp_path, cfg)
    p2 = tmp_path / "stage2.ckpt"
    torch.save({"state_dict": _xt_variant(s2.state_dict())}, p2)
    m = Stage2.load_from_checkpoint(str(p2), stage1_ckpt_fname=None, input_length=64,
                                    in_channels=6, n_classes=5, config=cfg)
    s2, m = s2.to(cuda).eval(), m.to(cuda).eval()
    gen = torch.Generator().manual_seed(0)
    s_l = torch.randint(0, 65, (4, s2.maskgit.num_tokens_l), generator=gen).to(cuda)
    y = torch.randint(0, 5, (4, 1), generator=gen).to(cuda)
    with torch.no_grad():
        a = s2.maskgit.transformer_l(s_l, class_condition=y)
        b = m.maskgit.transformer_l(s_l, class_condition=y)
    assert torch.equal(a, b)
