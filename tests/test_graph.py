"""hipGraph capture of the joint train step (bench.JointTrainer / timevqvae.hip.graph).

With the host-random choices switched off (layer dropout, classifier-free-guidance
condition drop -- both are drawn differently in graph mode by design), a graph replay
must reproduce the eager step bit for bit: every kernel is deterministic, conv / embedding
/ attention dropout masks are keyed on (device seed, site, call index in the step), and
the learning rate reaches the captured AdamW update through the device.
"""
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

pytestmark = pytest.mark.gpu


def _cfg():
    import bench
    cfg = bench.config(False)
    for k in ("prior_model_l", "prior_model_h"):
        cfg["MaskGIT"][k]["model_dropout"] = 0.0
        cfg["MaskGIT"][k]["p_unconditional"] = 0.0
    return cfg


def _state(tr):
    bufs = [b.detach().clone() for b in tr.s1.buffers() if b.is_floating_point()]
    return [tr.opt1.flat.clone(), tr.opt2.flat.clone(), tr.opt1.exp_avg_sq.clone()] + bufs


def _batch(dev, B=16, C=3, L=64):
    g = torch.Generator().manual_seed(5)
    x = torch.cumsum(0.1 * torch.randn(B, C, L, generator=g), -1)
    x = 2 * (x - x.amin(0, keepdim=True)) / (x.amax(0, keepdim=True) - x.amin(0, keepdim=True) + 1e-8) - 1
    return x.to(dev), torch.randint(0, 5, (B, 1), generator=g).to(dev)


def test_graph_replay_matches_eager(cuda):
    import bench
    batch = _batch(cuda)
    eager = bench.JointTrainer(cuda, 1, cfg=_cfg(), length=64, channels=3)
    losses_e = []
    for _ in range(4):
        o1, o2 = eager.step(batch)
        losses_e.append((float(o1["loss"].sum()), float(o2["loss"])))
    graphed = bench.JointTrainer(cuda, 1, cfg=_cfg(), length=64, channels=3)
    graphed.capture(batch)  # 2 eager warmup steps
    losses_g = []
    for _ in range(2):
        o1, o2 = graphed.step(batch)
        losses_g.append((float(o1["loss"].sum()), float(o2["loss"])))
    torch.cuda.synchronize()
    assert losses_g == losses_e[2:]
    for a, b in zip(_state(eager), _state(graphed)):
        assert torch.equal(a, b)


def test_graph_replays_advance(cuda):
    """Replays are real steps: parameters and dropout masks change from one to the next."""
    import bench
    batch = _batch(cuda)
    tr = bench.JointTrainer(cuda, 1, length=64, channels=3)
    tr.capture(batch)
    p0 = tr.opt1.flat.clone()
    o1, _ = tr.step(batch)
    l1 = float(o1["loss"].sum())
    p1 = tr.opt1.flat.clone()
    o1, _ = tr.step(batch)
    l2 = float(o1["loss"].sum())
    assert not torch.equal(p0, p1) and not torch.equal(p1, tr.opt1.flat)
    assert l1 != l2


def test_streams_match_single_stream(cuda):
    """The LF/HF branches on the side stream and the offloaded weight-gradient /
    codebook-statistics work change the schedule, never the result: eager steps with
    streams equal single-stream steps bit for bit (losses, parameters, optimizer state,
    codebooks), at the bench's shape family (config B dims, reduced batch), dropout on.
    test_graph_replay_matches_eager then covers the graphed multi-stream step."""
    import bench
    from timevqvae.hip import streams
    batch = _batch(cuda, B=32, C=6, L=256)
    prev = streams.ENABLED
    try:
        streams.ENABLED = False
        single = bench.JointTrainer(cuda, 1, cfg=_cfg(), length=256, channels=6)
        ls = [tuple(float(o["loss"].detach().sum()) for o in single.step(batch)) for _ in range(3)]
        streams.ENABLED = True
        multi = bench.JointTrainer(cuda, 1, cfg=_cfg(), length=256, channels=6)
        lm = [tuple(float(o["loss"].detach().sum()) for o in multi.step(batch)) for _ in range(3)]
    finally:
        streams.ENABLED = prev
    torch.cuda.synchronize()
    assert ls == lm
    for a, b in zip(_state(single), _state(multi)):
        assert torch.equal(a, b)


def test_pack_cache_matches_per_call_packing(cuda):
    """The per-step weight-pack cache (one batched repack at the scope's begin, convs read
    the arena) equals packing in every conv call bit for bit over several optimizer steps
    (the weights change between steps, so a stale pack would show), eager and graphed."""
    import bench
    from timevqvae.hip.conv import PackCache
    batch = _batch(cuda, B=32, C=6, L=256)
    ref = bench.JointTrainer(cuda, 1, cfg=_cfg(), length=256, channels=6)
    ref.packs = None
    lr = [tuple(float(o["loss"].detach().sum()) for o in ref.step(batch)) for _ in range(3)]
    cached = bench.JointTrainer(cuda, 1, cfg=_cfg(), length=256, channels=6)
    assert cached.packs is not None
    lc = [tuple(float(o["loss"].detach().sum()) for o in cached.step(batch)) for _ in range(3)]
    assert PackCache.entries() > 0
    torch.cuda.synchronize()
    assert lr == lc
    for a, b in zip(_state(ref), _state(cached)):
        assert torch.equal(a, b)
    # graphed with the cache == eager without it, two replays further
    ref2 = [tuple(float(o["loss"].detach().sum()) for o in ref.step(batch)) for _ in range(4)]
    g = bench.JointTrainer(cuda, 1, cfg=_cfg(), length=256, channels=6)
    for _ in range(3):
        g.step(batch)
    g.capture(batch)  # 2 more eager warmup steps, then capture
    lg = [tuple(float(o["loss"].detach().sum()) for o in g.step(batch)) for _ in range(2)]
    torch.cuda.synchronize()
    assert lg == ref2[2:]
    for a, b in zip(_state(ref), _state(g)):
        assert torch.equal(a, b)


def test_deferred_wgrad_reductions_match_immediate(cuda, monkeypatch):
    """Batching the conv weight-gradient split sums at the end of each band's backward
    (hip.conv.wgrad_deferred) gives the same gradients, parameters and optimizer state
    bit for bit as reducing after every conv, eager and graphed."""
    import bench
    batch = _batch(cuda, B=32, C=6, L=256)
    from timevqvae.hip import conv as hconv
    monkeypatch.setattr(hconv, "DEFER_WGRAD", False)
    ref = bench.JointTrainer(cuda, 1, cfg=_cfg(), length=256, channels=6)
    lr = [tuple(float(o["loss"].detach().sum()) for o in ref.step(batch)) for _ in range(7)]
    monkeypatch.setattr(hconv, "DEFER_WGRAD", True)
    d = bench.JointTrainer(cuda, 1, cfg=_cfg(), length=256, channels=6)
    ld = [tuple(float(o["loss"].detach().sum()) for o in d.step(batch)) for _ in range(3)]
    d.capture(batch)  # 2 eager warmup steps (deferral on), then capture
    ld += [tuple(float(o["loss"].detach().sum()) for o in d.step(batch)) for _ in range(2)]
    torch.cuda.synchronize()
    assert lr[:3] == ld[:3] and lr[5:] == ld[3:]
    for a, b in zip(_state(ref), _state(d)):
        assert torch.equal(a, b)
