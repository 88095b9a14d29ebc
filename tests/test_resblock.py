"""Fused ResBlock (csrc/tvq_resblock.hip, C in {8, 16, 32}; tvq_resblock_w8.hip, C = 64 on
the LF band's W = 8 maps; tvq_resblock_w8p.hip, the projection blocks 64 -> 128 and 128 -> 64
on those maps) against the per-op HIP path it
replaces (Snake -> conv -> BN+Snake -> conv+dropout+residual kernels, which the G3 goldens
pin to the reference): training forward (y, BN running stats), every gradient, the same
dropout mask, and the eval forward.  Tolerance: rel 2e-5 of each tensor's max (different
summation order of the same fp32 arithmetic)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = [(8, 8, 64), (8, 16, 32), (4, 16, 16), (16, 8, 32), (3, 32, 16), (2, 32, 32),
          (2, 16, 64), (5, 8, 16), (8, 64, 8), (3, 64, 8), (300, 64, 8)]


def _block(C, drop, seed=0, Co=None):
    from timevqvae.models.vq_vae import ResBlock
    torch.manual_seed(seed)
    m = ResBlock(C, Co or C, False, dropout=drop)
    with torch.no_grad():
        for p in m.parameters():
            p.copy_(torch.randn_like(p) * (0.3 if p.dim() > 1 else 0.5))
        m.convs[0].a.uniform_(0.3, 0.8)
        m.convs[3].a.uniform_(0.3, 0.8)
        m.convs[2].running_mean.normal_()
        m.convs[2].running_var.uniform_(0.5, 2.0)
    return m.cuda()


def _run(m, x, fused, train=True):
    from timevqvae.hip import resblock, rng
    prev = resblock.ENABLED
    resblock.ENABLED = fused
    try:
        rng._calls[0] = 0
        m.train(train)
        for p in m.parameters():
            p.grad = None
        xx = x.clone().requires_grad_(train)
        if train:
            y = m(xx)
            gy = torch.cos(torch.arange(y.numel(), device=y.device, dtype=torch.float32)).view_as(y)
            y.backward(gy)
            grads = {n: p.grad.clone() for n, p in m.named_parameters()}
            grads["x"] = xx.grad.clone()
        else:
            with torch.no_grad():
                y = m(xx)
            grads = {}
        bufs = {n: b.clone() for n, b in m.named_buffers()}
        return y.detach(), grads, bufs
    finally:
        resblock.ENABLED = prev


def _close(a, b, name, rel=2e-5):
    scale = b.abs().max().item() + 1e-6
    err = (a - b).abs().max().item()
    assert err <= rel * scale, f"{name}: max err {err:.3e} vs scale {scale:.3e}"


@pytest.mark.parametrize("B,C,W", SHAPES)
@pytest.mark.parametrize("drop", [0.0, 0.3])
def test_fused_resblock_train_matches_per_op(B, C, W, drop):
    from timevqvae.hip import resblock
    x = torch.randn(B, C, 3, W, device="cuda")
    assert resblock.supported(x, C, C)
    m1 = _block(C, drop)
    m2 = _block(C, drop)
    m2._site = m1._site  # same dropout call site -> same mask stream
    y1, g1, b1 = _run(m1, x, fused=False)
    y2, g2, b2 = _run(m2, x, fused=True)
    _close(y2, y1, "y")
    for k in g1:
        if k == "convs.1.bias":
            # conv1's bias feeds a BatchNorm: its true gradient is 0 (rounding noise only)
            tol = 2e-5 * g1["convs.1.weight"].abs().max().item()
            assert (g2[k] - g1[k]).abs().max().item() <= tol, k
            continue
        _close(g2[k], g1[k], k)
    for k in b1:
        if b1[k].is_floating_point():
            _close(b2[k], b1[k], k)
        else:
            assert torch.equal(b2[k], b1[k]), k
    if drop > 0:  # the dropout really dropped, identically: zero pattern of y - x agrees
        assert torch.equal((y1 - x) == 0, (y2 - x) == 0)
        assert ((y2 - x) == 0).float().mean().item() > 0.2


PAIR_SHAPES = [(8, 8, 64), (8, 16, 32), (4, 16, 16), (3, 32, 16), (2, 32, 32), (5, 8, 16),
               (8, 64, 8), (3, 64, 8), (256, 64, 8),
               (32, 32, 16), (256, 32, 16)]  # B % 16 == 0: RB<32,16> external weight gradients


def _run_pair(ms, x, paired):
    from timevqvae.hip import resblock, rng
    from timevqvae.hip._native import plan_trace
    from timevqvae.models.vq_vae import run_layers
    prev = resblock.PAIR_ENABLED
    resblock.PAIR_ENABLED = paired
    try:
        rng._calls[0] = 0
        for m in ms:
            m.train(True)
            for p in m.parameters():
                p.grad = None
        xx = x.clone().requires_grad_(True)
        with plan_trace() as tr:
            y = run_layers(ms, xx, lambda layer, v: layer(v))
            gy = torch.cos(torch.arange(y.numel(), device=y.device, dtype=torch.float32)).view_as(y)
            y.backward(gy)
        torch.cuda.synchronize()
        grads = {f"{i}.{n}": p.grad.clone() for i, m in enumerate(ms)
                 for n, p in m.named_parameters()}
        grads["x"] = xx.grad.clone()
        bufs = {f"{i}.{n}": b.clone() for i, m in enumerate(ms) for n, b in m.named_buffers()}
        return y.detach(), grads, bufs, tr.lines
    finally:
        resblock.PAIR_ENABLED = prev


@pytest.mark.parametrize("B,C,W", PAIR_SHAPES)
@pytest.mark.parametrize("drop", [0.0, 0.3])
def test_resblock_pair_bitwise_equals_two_blocks(B, C, W, drop):
    """rb_fwd21 / rb_bwd12 and, C = 64, w8_fwd21 / w8_bwd12 (block 1's second kernel and
    block 2's first in one launch, the activation handed over in registers) compute exactly what the two blocks' separate
    launches do: y, every gradient and the BN running statistics bitwise equal."""
    from timevqvae.hip import resblock
    x = torch.randn(B, C, 3, W, device="cuda")
    assert resblock.pair_supported(x)
    ms_a = [_block(C, drop, seed=1), _block(C, drop, seed=2)]
    ms_b = [_block(C, drop, seed=1), _block(C, drop, seed=2)]
    for ma, mb in zip(ms_a, ms_b):
        mb._site = ma._site
    ya, ga, ba, ta = _run_pair(ms_a, x, paired=False)
    yb, gb, bb, tb = _run_pair(ms_b, x, paired=True)
    k = "w8" if C == 64 else "rb"
    assert not any("fwd21" in t for t in ta)
    assert any(t.startswith(f"{k}_fwd21 C{C} W{W}") for t in tb), tb
    assert any(t.startswith(f"{k}_bwd12 C{C} W{W}") for t in tb), tb
    assert torch.equal(ya, yb)
    for k in ga:
        assert torch.equal(ga[k], gb[k]), k
    for k in ba:
        assert torch.equal(ba[k], bb[k]), k


def test_resblock_pair_not_used_in_eval():
    x = torch.randn(4, 16, 3, 32, device="cuda")
    ms = [_block(16, 0.0, seed=1), _block(16, 0.0, seed=2)]
    from timevqvae.hip._native import plan_trace
    from timevqvae.models.vq_vae import run_layers
    for m in ms:
        m.eval()
    with torch.no_grad(), plan_trace() as tr:
        run_layers(ms, x, lambda layer, v: layer(v))
    assert not any("fwd21" in t for t in tr.lines)


def test_fused_resblock_w8_eval_packed_and_unpacked():
    """The C = 64 eval kernel reads packed weights inside a pack-cache scope and the raw
    (n, c, tap) weights outside one: the same results either way."""
    from timevqvae.hip.conv import PackCache
    from timevqvae.hip._native import plan_trace
    x = torch.randn(6, 64, 3, 8, device="cuda")
    m = _block(64, 0.3).eval()
    with torch.no_grad(), plan_trace() as tr:
        y1 = m(x)
        with PackCache(x.device).scope():
            y2 = m(x)
            y3 = m(x)
        torch.cuda.synchronize()
    assert tr.has("w8_eval C64 W8 B6 packed=0") and tr.has("w8_eval C64 W8 B6 packed=1"), tr.lines
    _close(y2, y1, "packed vs raw")
    assert torch.equal(y2, y3)


@pytest.mark.parametrize("B,C,W", SHAPES)
def test_fused_resblock_eval_matches_per_op(B, C, W):
    x = torch.randn(B, C, 3, W, device="cuda")
    m = _block(C, 0.3)
    y1, _, _ = _run(m, x, fused=False, train=False)
    y2, _, _ = _run(m, x, fused=True, train=False)
    _close(y2, y1, "y eval")


def test_fused_resblock_declines_unsupported_shapes():
    from timevqvae.hip import resblock
    assert resblock.supported(torch.empty(2, 64, 3, 8, device="cuda"), 64, 64)
    assert not resblock.supported(torch.empty(2, 64, 3, 16, device="cuda"), 64, 64)
    assert not resblock.supported(torch.empty(2, 128, 3, 8, device="cuda"), 128, 128)
    assert not resblock.supported(torch.empty(2, 32, 3, 64, device="cuda"), 32, 32)
    assert not resblock.supported(torch.empty(2, 4, 3, 32, device="cuda"), 4, 4)
    assert not resblock.supported(torch.empty(2, 8, 3, 20, device="cuda"), 8, 8)
    assert not resblock.supported(torch.empty(2, 8, 3, 128, device="cuda"), 8, 8)
    assert not resblock.supported(torch.empty(2, 8, 3, 32, device="cuda"), 8, 16)


PROJ_SHAPES = [(8, 64, 128), (3, 128, 64), (256, 64, 128), (256, 128, 64), (37, 64, 128)]


@pytest.mark.parametrize("B,Ci,Co", PROJ_SHAPES)
@pytest.mark.parametrize("drop", [0.0, 0.3])
def test_fused_proj_resblock_train_matches_per_op(B, Ci, Co, drop):
    """The projection block (1x1 proj on the skip) at the LF band's W = 8: every gradient
    (conv, proj, BN, Snake), the running statistics and the dropout mask against the
    per-op path, and the fused kernels' plan names."""
    from timevqvae.hip import resblock
    from timevqvae.hip._native import plan_trace
    x = torch.randn(B, Ci, 3, 8, device="cuda")
    assert resblock.proj_supported(x, Ci, Co)
    m1 = _block(Ci, drop, Co=Co)
    m2 = _block(Ci, drop, Co=Co)
    m2._site = m1._site
    y1, g1, b1 = _run(m1, x, fused=False)
    with plan_trace() as tr:
        y2, g2, b2 = _run(m2, x, fused=True)
        torch.cuda.synchronize()
    assert tr.has(f"w8p_fwd Ci{Ci} Co{Co} B{B}") and tr.has(f"w8p_bwd Ci{Ci} Co{Co} B{B}"), tr.lines
    _close(y2, y1, "y")
    for k in g1:
        if k == "convs.1.bias":
            tol = 2e-5 * g1["convs.1.weight"].abs().max().item()
            assert (g2[k] - g1[k]).abs().max().item() <= tol, k
            continue
        _close(g2[k], g1[k], k)
    for k in b1:
        if b1[k].is_floating_point():
            _close(b2[k], b1[k], k)
        else:
            assert torch.equal(b2[k], b1[k]), k
    if drop > 0:
        # the dropout really dropped (y = proj(x) there); that it dropped the same elements
        # is what the y comparison above shows (a different mask moves y by O(1))
        r = torch.nn.functional.conv2d(x, m1.proj.weight, m1.proj.bias)
        tol = 1e-4 * r.abs().max().item()
        assert ((y2 - r).abs() < tol).float().mean().item() > 0.2
        assert ((y1 - r).abs() < tol).float().mean().item() > 0.2


@pytest.mark.parametrize("B,Ci,Co", PROJ_SHAPES)
def test_fused_proj_resblock_eval_matches_per_op(B, Ci, Co):
    from timevqvae.hip.conv import PackCache
    from timevqvae.hip._native import plan_trace
    x = torch.randn(B, Ci, 3, 8, device="cuda")
    m = _block(Ci, 0.3, Co=Co)
    y1, _, _ = _run(m, x, fused=False, train=False)
    with plan_trace() as tr:
        y2, _, _ = _run(m, x, fused=True, train=False)
        with PackCache(x.device).scope(), torch.no_grad():
            y3 = m.eval()(x)
        torch.cuda.synchronize()
    assert tr.has(f"w8p_eval Ci{Ci} Co{Co} B{B} packed=0"), tr.lines
    assert tr.has(f"w8p_eval Ci{Ci} Co{Co} B{B} packed=1"), tr.lines
    _close(y2, y1, "y eval")
    _close(y3, y1, "y eval packed")


def test_fused_proj_resblock_declines_unsupported_shapes():
    from timevqvae.hip import resblock
    assert resblock.proj_supported(torch.empty(2, 64, 3, 8, device="cuda"), 64, 128)
    assert resblock.proj_supported(torch.empty(2, 128, 3, 8, device="cuda"), 128, 64)
    assert not resblock.proj_supported(torch.empty(2, 64, 3, 8, device="cuda"), 64, 64)
    assert not resblock.proj_supported(torch.empty(2, 16, 3, 32, device="cuda"), 16, 128)
    assert not resblock.proj_supported(torch.empty(2, 64, 3, 16, device="cuda"), 64, 128)
    assert not resblock.proj_supported(torch.empty(2, 32, 3, 8, device="cuda"), 32, 64)
