"""Per-kernel numerics: each HIP op vs the plain PyTorch fp32 CPU op (forward and
backward).  Tolerance: rel-L2 <= 1e-5 (fp32 reassociation only), max-abs scaled."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return float((a - b).norm() / (b.norm() + 1e-30))


def close(a, b, tol=1e-5, what=""):
    r = rel(a, b)
    assert r <= tol, f"{what}: rel-L2 {r:.3e} > {tol}"


def _grads(fn, inputs):
    outs = fn(*inputs)
    g = torch.randn_like(outs)
    outs.backward(g)
    return outs, [t.grad for t in inputs], g


@pytest.fixture
def conv_path(monkeypatch):
    """Select the conv engine: the default per-shape choice, the halo-tile kernel
    wherever it fits, the staged GEMMs with packed weights (32x32-MFMA wide tile where
    eligible; "tap" = the 16x16 tap-major kernel only), or the staged GEMM reading the
    weights in place; "no_s2" = the default choice without the stride-2 small-channel
    kernels (conv_s2f / conv_s2t / conv_wgrad_s2)."""
    from timevqvae.hip import conv as conv_mod
    from timevqvae.hip._native import value
    prev = value("tvq_conv_config", -1)

    def select(path):
        monkeypatch.setattr(conv_mod, "USE_WORKSPACE", path != "gemm_raw")
        value("tvq_conv_config", {"default": 3, "halo": 7, "tap": 8, "no_s2": 3 | 512 | 1024}.get(path, 0))

    yield select
    value("tvq_conv_config", prev)


def _run_both(fn_hip, fn_ref, shapes, cuda, seed=0):
    gen = torch.Generator().manual_seed(seed)
    cpu = [torch.randn(s, generator=gen).requires_grad_(True) for s in shapes]
    dev = [t.detach().to(cuda).requires_grad_(True) for t in cpu]
    out_c = fn_ref(*cpu)
    g = torch.randn(out_c.shape, generator=gen)
    out_c.backward(g)
    out_d = fn_hip(*dev)
    out_d.backward(g.to(cuda))
    torch.cuda.synchronize()
    return out_c, out_d, cpu, dev


@pytest.mark.parametrize("B,Ci,Co,W,kind", [
    (4, 12, 4, 257, "enc"), (3, 8, 16, 64, "enc"), (2, 32, 64, 16, "enc"),
    # stride-2 small-channel kernels: 16 channels, channels not a multiple of 4, ragged widths
    (2, 16, 16, 128, "enc"), (2, 6, 5, 70, "enc"), (3, 4, 8, 130, "enc"),
    (2, 4, 4, 63, "enc"),  # replicate-canvas columns W, W+1 across a segment: canvas + fold
    (4, 8, 8, 64, "res"), (2, 64, 128, 8, "res"), (2, 16, 128, 32, "res"), (3, 128, 16, 32, "res"),
    (2, 64, 128, 8, "proj"), (5, 3, 7, 33, "res"),
    # the wide-map weight-gradient kernel (conv_wgrad_t32_kernel): the HF 128 -> 128 conv,
    # an uneven last position split (37 images), a 64-wide map
    (2, 128, 128, 32, "res"), (37, 128, 128, 32, "res"), (3, 32, 64, 64, "res"),
])
@pytest.mark.parametrize("path", ["default", "halo", "gemm", "tap", "gemm_raw", "no_s2"])
def test_conv2d(B, Ci, Co, W, kind, path, cuda, conv_path):
    from timevqvae.hip.conv import conv2d
    conv_path(path)
    if kind == "enc":
        KH, KW, SW, rep = 3, 4, 2, True
    elif kind == "res":
        KH, KW, SW, rep = 3, 3, 1, False
    else:
        KH, KW, SW, rep = 1, 1, 1, False

    def ref(x, w, b):
        xp = F.pad(x, (1, 1, 1, 1), mode="replicate") if rep else x
        pad = (0, 0) if rep else (KH // 2, (KW - 1) // 2)
        return F.conv2d(xp, w, b, stride=(1, SW), padding=pad)

    def hip(x, w, b):
        return conv2d(x, w, b, stride_w=SW, replicate=rep)

    oc, od, c, d = _run_both(hip, ref, [(B, Ci, 3, W), (Co, Ci, KH, KW), (Co,)], cuda)
    close(od, oc, what="fwd")
    for i, n in enumerate(("dx", "dw", "db")):
        close(d[i].grad, c[i].grad, what=n)


@pytest.mark.parametrize("B,Ci,Co,W", [(4, 64, 32, 8), (2, 8, 4, 64), (3, 4, 12, 128), (2, 12, 12, 256),
                                        (2, 128, 128, 16), (2, 16, 16, 40), (3, 5, 7, 37)])
@pytest.mark.parametrize("path", ["default", "halo", "gemm", "tap", "gemm_raw", "no_s2"])
def test_conv_transpose2d(B, Ci, Co, W, path, cuda, conv_path):
    from timevqvae.hip.conv import conv_transpose2d
    conv_path(path)

    def ref(x, w, b):
        return F.conv_transpose2d(x, w, b, stride=(1, 2), padding=(1, 1))

    oc, od, c, d = _run_both(lambda x, w, b: conv_transpose2d(x, w, b), ref,
                             [(B, Ci, 3, W), (Ci, Co, 3, 4), (Co,)], cuda)
    close(od, oc, what="fwd")
    for i, n in enumerate(("dx", "dw", "db")):
        close(d[i].grad, c[i].grad, what=n)


@pytest.mark.parametrize("B,Ci,Co", [(8, 128, 256), (20, 256, 128)])  # the HF prior's Upscale
def test_conv1d_k3(B, Ci, Co, cuda):
    from timevqvae.hip.conv import conv2d
    oc, od, c, d = _run_both(lambda x, w, b: conv2d(x, w, b), lambda x, w, b: F.conv1d(x, w, b, padding=1),
                             [(B, Ci, 96), (Co, Ci, 3), (Co,)], cuda)
    close(od, oc, what="fwd")
    for i, n in enumerate(("dx", "dw", "db")):
        close(d[i].grad, c[i].grad, what=n)


def test_conv_residual_dropout(cuda):
    """Fused epilogue: out = residual + Dropout(conv + b); mask regenerated in backward."""
    from timevqvae.hip.conv import conv2d
    gen = torch.Generator().manual_seed(1)
    x = torch.randn(4, 16, 3, 32, generator=gen).to(cuda).requires_grad_(True)
    w = torch.randn(16, 16, 3, 3, generator=gen).to(cuda).requires_grad_(True)
    r = torch.randn(4, 16, 3, 32, generator=gen).to(cuda).requires_grad_(True)
    y = conv2d(x, w, None, residual=r, drop_p=0.3, site=12345)
    base = conv2d(x.detach(), w.detach(), None)
    v = (y - r).detach()
    kept = v != 0
    frac = kept.float().mean().item()
    assert 0.6 < frac < 0.8, frac
    torch.testing.assert_close(v[kept], (base / 0.7)[kept], rtol=1e-5, atol=1e-5)
    g = torch.randn_like(y)
    y.backward(g)
    torch.testing.assert_close(r.grad, g)
    # dx = dgrad(g * mask / 0.7)
    x2 = x.detach().clone().requires_grad_(True)
    conv2d(x2, w.detach(), None).backward(g * kept / 0.7)
    torch.testing.assert_close(x.grad, x2.grad, rtol=1e-5, atol=1e-5)


# chunked form (C < 32) and the whole-channel form (C >= 32, B*3W <= 24576), including the
# step's LF (256, 64, 3, 8) and HF (256, 128, 3, 32) shapes
# (plus the step's small-channel EncBlock / DecBlock outputs (256, 4|8|16, 3, 128|64|32))
@pytest.mark.parametrize("B,C,W,snake_on", [(8, 16, 32, True), (4, 4, 128, True), (16, 128, 8, True),
                                            (8, 256, 96, False), (256, 64, 8, True),
                                            (256, 128, 32, True), (64, 32, 16, False),
                                            (256, 4, 128, True), (256, 8, 64, True),
                                            (256, 16, 32, True), (256, 12, 128, False),
                                            (100, 8, 64, True)])
def test_bn_snake_train(B, C, W, snake_on, cuda):
    from timevqvae.hip.norm import bn_snake
    bn_c = torch.nn.BatchNorm2d(C).train()
    with torch.no_grad():
        bn_c.weight.uniform_(0.5, 1.5)
        bn_c.bias.uniform_(-0.2, 0.2)
        bn_c.running_var.uniform_(0.5, 1.5)
    bn_d = torch.nn.BatchNorm2d(C).to(cuda).train()
    bn_d.load_state_dict(bn_c.state_dict())
    a_c = torch.empty(C).uniform_(0.2, 0.5).requires_grad_(True)
    a_d = a_c.detach().to(cuda).requires_grad_(True)
    gen = torch.Generator().manual_seed(2)
    x_c = (torch.randn(B, C, 3, W, generator=gen) * 2 + 0.5).requires_grad_(True)
    x_d = x_c.detach().to(cuda).requires_grad_(True)

    def ref(x):
        s = bn_c(x)
        if snake_on:
            a = a_c.view(1, C, 1, 1)
            s = s + (1 / a) * torch.sin(a * s) ** 2
        return s

    y_c = ref(x_c)
    g = torch.randn(y_c.shape, generator=gen)
    y_c.backward(g)
    y_d = bn_snake(x_d, bn_d, a_d if snake_on else None)
    y_d.backward(g.to(cuda))
    close(y_d, y_c, what="fwd")
    close(x_d.grad, x_c.grad, tol=2e-5, what="dx")
    close(bn_d.weight.grad, bn_c.weight.grad, what="dw")
    close(bn_d.bias.grad, bn_c.bias.grad, what="db")
    if snake_on:
        close(a_d.grad, a_c.grad, tol=2e-5, what="da")
    close(bn_d.running_mean, bn_c.running_mean, what="running_mean")
    close(bn_d.running_var, bn_c.running_var, what="running_var")
    assert int(bn_d.num_batches_tracked) == int(bn_c.num_batches_tracked)


def test_bn_eval(cuda):
    from timevqvae.hip.norm import bn_snake
    bn_c = torch.nn.BatchNorm2d(32).eval()
    with torch.no_grad():
        bn_c.running_mean.uniform_(-1, 1)
        bn_c.running_var.uniform_(0.5, 2)
        bn_c.weight.uniform_(0.5, 1.5)
    bn_d = torch.nn.BatchNorm2d(32).to(cuda).eval()
    bn_d.load_state_dict(bn_c.state_dict())
    x = torch.randn(4, 32, 3, 16)
    a = torch.empty(32).uniform_(0.2, 0.5)
    with torch.no_grad():
        s = bn_c(x)
        ref = s + (1 / a.view(1, -1, 1, 1)) * torch.sin(a.view(1, -1, 1, 1) * s) ** 2
        got = bn_snake(x.to(cuda), bn_d, a.to(cuda))
    close(got, ref, what="eval bn+snake")


def test_snake(cuda):
    from timevqvae.hip.norm import snake
    C = 24
    a_c = torch.empty(C).uniform_(0.2, 0.5).requires_grad_(True)
    a_d = a_c.detach().to(cuda).requires_grad_(True)
    oc, od, c, d = _run_both(lambda x: snake(x, a_d),
                             lambda x: x + (1 / a_c.view(1, C, 1, 1)) * torch.sin(a_c.view(1, C, 1, 1) * x) ** 2,
                             [(6, C, 3, 40)], cuda)
    close(od, oc, what="fwd")
    close(d[0].grad, c[0].grad, what="dx")
    close(a_d.grad, a_c.grad, tol=2e-5, what="da")


@pytest.mark.parametrize("T", [128, 256])
def test_stft_encode_vs_golden(T, cuda):
    from conftest import golden
    from timevqvae.hip.signal import stft_encode
    g = golden("g2_stft.npz")
    x = torch.from_numpy(g[f"x_T{T}"]).to(cuda)
    o = stft_encode(x, raw=True, enc_l=True, enc_h=True, tgt_l=True, tgt_h=True)
    for k, gk in (("raw", "xf"), ("enc_l", "lf_copy"), ("enc_h", "hf_copy"), ("tgt_l", "x_l"), ("tgt_h", "x_h")):
        np.testing.assert_allclose(o[k].cpu().numpy(), g[f"{gk}_T{T}"], rtol=1e-5, atol=1e-6, err_msg=k)


@pytest.mark.parametrize("T,band", [(128, "lf"), (256, "hf"), (256, "lf"), (128, "all")])
def test_istft_decode(T, band, cuda):
    """band-mask + iSTFT + Upsample(T, linear): fwd vs golden/oracle, bwd vs autograd of the oracle."""
    from conftest import golden
    from oracle import tvq_oracle as O
    from timevqvae.hip.signal import istft_decode
    g = golden("g2_stft.npz")
    img = torch.from_numpy(g[f"dec_img_T{T}"])
    mask = {"lf": O.band_lf, "hf": O.band_hf, "all": lambda z: z}[band]
    img_c = img.clone().requires_grad_(True)
    Tout = T if band != "all" else 2 * T - 1
    y_c = O.linear_interp(O.istft4(mask(img_c), 6), Tout)
    if band != "all":
        np.testing.assert_allclose(O.istft4(mask(img), 6).numpy(), g[f"dec_istft_{band}_T{T}"], rtol=1e-5, atol=1e-6)
    img_d = img.to(cuda).requires_grad_(True)
    y_d = istft_decode(img_d, 6, band, Tout)
    gy = torch.randn(y_c.shape)
    y_c.backward(gy)
    y_d.backward(gy.to(cuda))
    close(y_d, y_c, what="fwd")
    close(img_d.grad, img_c.grad, what="bwd")


@pytest.mark.parametrize("M,K,N,res", [(1536, 256, 256, True), (100, 33, 70, False), (6400, 128, 513, False)])
def test_linear(M, K, N, res, cuda):
    from timevqvae.hip.linear import linear
    shapes = [(M, K), (N, K), (N,)] + ([(M, N)] if res else [])

    def ref(x, w, b, r=None):
        y = F.linear(x, w, b)
        return y + r if r is not None else y

    def hip(x, w, b, r=None):
        return linear(x, w, b, residual=r)

    oc, od, c, d = _run_both(hip, ref, shapes, cuda)
    close(od, oc, what="fwd")
    for i in range(len(shapes)):
        close(d[i].grad, c[i].grad, what=f"grad{i}")


@pytest.mark.parametrize("M,N,K", [(25600, 128, 128), (300, 512, 128), (97, 32, 256), (1000, 64, 32),
                                   (130, 600, 64), (64, 96, 512), (7, 3, 4), (2000, 384, 128)])
@pytest.mark.parametrize("epi", ["plain", "bias_gelu_pre", "res_rmod_acc"])
def test_gemm_nt_epilogues(M, N, K, epi, cuda):
    """C = epi(alpha A W^T) on the MFMA NT path (A, W k-contiguous) against torch fp32."""
    from timevqvae.hip.linear import gemm
    gen = torch.Generator().manual_seed(M + N + K)
    A = torch.randn(M, K, generator=gen)
    W = torch.randn(N, K, generator=gen) / K ** 0.5
    b = torch.randn(N, generator=gen)
    R = torch.randn(24, N, generator=gen)
    C0 = torch.randn(M, N, generator=gen)
    ref = 0.5 * (A.double() @ W.double().t())
    kw = {}
    if epi == "bias_gelu_pre":
        pre_ref = ref + b.double()
        ref = F.gelu(pre_ref)
        pre = torch.empty(M, N, device=cuda)
        kw = dict(bias=b.to(cuda), act=1, pre=pre)
    elif epi == "res_rmod_acc":
        ref = ref + R.double()[torch.arange(M) % 24] + C0.double()
        kw = dict(R=R.to(cuda), ldr=N, rmod=24, accumulate=True)
    out = C0.to(cuda) if epi == "res_rmod_acc" else None
    y = gemm(A.to(cuda), K, 1, W.to(cuda), 1, K, M, N, K, out=out, ldc=N if out is not None else None,
             alpha=0.5, **kw)
    err = float((y.cpu().double() - ref).norm() / ref.norm())
    assert err < 2e-6, err
    if epi == "bias_gelu_pre":
        assert float((pre.cpu().double() - pre_ref).norm() / pre_ref.norm()) < 2e-6


@pytest.mark.parametrize("M,N,K,kind", [(6400, 128, 128, "nn"), (6144, 128, 512, "nn"), (501, 70, 36, "nn"),
                                        (128, 128, 6400, "tn"), (512, 128, 6144, "tn"),
                                        (128, 256, 24576, "tn"), (33, 70, 1001, "tn"), (256, 256, 1536, "tn")])
def test_gemm_nn_tn(M, N, K, kind, cuda):
    """dX = dY W (nn: B n-contiguous) and dW (+)= dY^T X (tn: split over rows, slabs summed
    in order) against torch fp64; tn accumulates into an existing buffer (the flat grad)."""
    from timevqvae.hip.linear import gemm
    gen = torch.Generator().manual_seed(M * 7 + N + K)
    C0 = torch.randn(M, N, generator=gen)
    if kind == "nn":
        A = torch.randn(M, K, generator=gen)
        B = torch.randn(K, N, generator=gen) / K ** 0.5
        y = gemm(A.to(cuda), K, 1, B.to(cuda), N, 1, M, N, K)
        ref = A.double() @ B.double()
    else:
        A = torch.randn(K, M, generator=gen) / K ** 0.5
        B = torch.randn(K, N, generator=gen)
        y = gemm(A.to(cuda), 1, M, B.to(cuda), N, 1, M, N, K, out=C0.to(cuda), ldc=N, accumulate=True)
        ref = A.double().t() @ B.double() + C0.double()
    err = float((y.cpu().double() - ref).norm() / ref.norm())
    assert err < 2e-6, err


@pytest.mark.parametrize("case", ["lf_prior", "hf_prior", "ragged_chunked"])
def test_wgrad_group(case, cuda):
    """tvq_wgrad_group: dW_i += dY_i^T X_i for a list of Linear layers in one launch, the
    outputs being views into one flat gradient buffer (as FusedAdamW keeps them), against
    torch fp64; run twice from the same start, bitwise equal (fixed-order sums).
    lf_prior: the LF prior's 16 weight gradients (4 layers x [q|k|v 384x128, out, ff1,
    ff2 128x128], 6400 tokens, 64x64 tiles); hf_prior: the HF prior's (dim 32: 32x32 tiles,
    24832 tokens); ragged_chunked: 30 odd shapes (two chunks of <= 24 descriptors), mixed
    token counts and padded leading dimensions."""
    from timevqvae.hip import wgrad
    gen = torch.Generator().manual_seed(7)
    if case == "lf_prior":
        shapes = [(384, 128, 6400), (128, 128, 6400), (128, 128, 6400), (128, 128, 6400)] * 4
    elif case == "hf_prior":
        shapes = [(192, 32, 24832), (32, 64, 24832), (32, 32, 24832), (32, 32, 24832)]
    else:
        shapes = [(33 + 7 * i, 70 - 2 * i, 1001 + 97 * i) for i in range(30)]
    flat = torch.randn(sum(m * n for m, n, _ in shapes), generator=gen)
    recs, refs, off = [], [], 0
    for i, (M, N, K) in enumerate(shapes):
        pad = 3 if case == "ragged_chunked" and i % 2 else 0
        dy = torch.randn(K, M + pad, generator=gen) / K ** 0.5
        x = torch.randn(K, N + pad, generator=gen)
        c0 = flat[off:off + M * N].view(M, N)
        refs.append(dy[:, :M].double().t() @ x[:, :N].double() + c0.double())
        recs.append((dy.to(cuda), M + pad, x.to(cuda), N + pad, (off, M * N), N, M, N, K))
        off += M * N
    outs = []
    for _ in range(2):
        fd = flat.to(cuda)
        wgrad.launch([r[:4] + (fd[r[4][0]:r[4][0] + r[4][1]],) + r[5:] for r in recs])
        outs.append(fd.cpu())
    assert torch.equal(outs[0], outs[1])
    off = 0
    for (M, N, K), ref in zip(shapes, refs):
        y = outs[0][off:off + M * N].view(M, N).double()
        off += M * N
        err = float((y - ref).norm() / ref.norm())
        assert err < 2e-6, (M, N, K, err)


@pytest.mark.parametrize("case", ["lf_prior", "hf_prior", "ragged_chunked"])
def test_wgrad_group_bias(case, cuda):
    """tvq_wgrad_group_bias: the Linear bias gradients db_i += column sums of dY_i taken in
    the grouped weight-gradient launch (every other record has one; the rest keep
    db = NULL), against torch fp64; dW unchanged bit for bit by the bias rows riding
    along; run twice, bitwise equal."""
    from timevqvae.hip import wgrad
    gen = torch.Generator().manual_seed(5)
    if case == "lf_prior":
        shapes = [(384, 128, 6400), (128, 128, 6400), (128, 128, 6400), (128, 128, 6400)] * 2
    elif case == "hf_prior":
        shapes = [(192, 32, 24832), (32, 64, 24832), (32, 32, 24832), (64, 32, 24832)]
    else:
        shapes = [(33 + 7 * i, 70 - 2 * i, 1001 + 97 * i) for i in range(28)]
    nw = sum(m * n for m, n, _ in shapes)
    flat = torch.randn(nw + sum(m for m, _, _ in shapes), generator=gen)
    recs, off, boff = [], 0, nw
    for i, (M, N, K) in enumerate(shapes):
        pad = 3 if case == "ragged_chunked" and i % 3 == 1 else 0
        dy = torch.randn(K, M + pad, generator=gen) / K ** 0.5
        x = torch.randn(K, N + pad, generator=gen)
        recs.append((dy, M + pad, x, N + pad, off, boff if i % 2 == 0 else None, M, N, K))
        off += M * N
        boff += M
    outs = []
    for with_bias in (True, True, False):
        fd = flat.to(cuda)
        rr = []
        for dy, ldy, x, ldx, o, bo, M, N, K in recs:
            r = (dy.to(cuda), ldy, x.to(cuda), ldx, fd[o:o + M * N], N, M, N, K)
            if with_bias:
                r = r + (fd[bo:bo + M] if bo is not None else None,)
            rr.append(r)
        wgrad.launch(rr)
        outs.append(fd.cpu())
    assert torch.equal(outs[0], outs[1])
    assert torch.equal(outs[0][:nw], outs[2][:nw])  # dW: the bias rows change nothing
    for dy, ldy, x, ldx, o, bo, M, N, K in recs:
        if bo is None:
            continue
        ref = dy[:, :M].double().sum(0) + flat[bo:bo + M].double()
        err = float((outs[0][bo:bo + M].double() - ref).abs().max() / ref.abs().max())
        assert err < 2e-6, (M, N, K, err)
    # the records without a bias output leave their bias rows alone
    keep = torch.ones(flat.numel(), dtype=torch.bool)
    for dy, ldy, x, ldx, o, bo, M, N, K in recs:
        if bo is not None:
            keep[bo:bo + M] = False
    keep[:nw] = False
    assert torch.equal(outs[0][keep], flat[keep])


def test_wgrad_group_forms_bitwise_equal(cuda):
    """The wide 128x64 form (16-byte-aligned operands) and the 64x64 form (the same data
    one float off alignment) sum every element in the same order: equal bit for bit, so a
    weight gradient does not depend on the allocator's alignment or on its group."""
    from timevqvae.hip import wgrad
    gen = torch.Generator().manual_seed(11)
    M, N, K = 384, 128, 6400
    dy = torch.randn(K, M, generator=gen).to(cuda)
    x = torch.randn(K, N, generator=gen).to(cuda)
    buf = torch.empty(K * M + 1, device=cuda)
    dy_off = buf[1:].view(K, M)
    dy_off.copy_(dy)
    outs = []
    for a in (dy, dy_off):
        dw = torch.zeros(M, N, device=cuda)
        wgrad.launch([(a, M, x, N, dw, N, M, N, K)])
        outs.append(dw)
    assert torch.equal(outs[0], outs[1])


def test_wgrad_group_deferral_keeps_order(cuda):
    """Inside wgrad.grouped(), weight_grad records are issued at the scope's exit; a record
    whose output overlaps a pending one flushes the pending ones first, so two
    accumulations into one buffer keep their order (result equals back-to-back tvq_gemm)."""
    from timevqvae.hip import wgrad
    gen = torch.Generator().manual_seed(3)
    M, N, K = 128, 128, 6400
    dys = [torch.randn(K, M, generator=gen).to(cuda) for _ in range(3)]
    xs = [torch.randn(K, N, generator=gen).to(cuda) for _ in range(3)]
    dw = torch.zeros(2, M, N, device=cuda)
    with wgrad.grouped():
        assert wgrad.defer(dys[0], M, xs[0], N, dw[0], N, M, N, K)
        assert wgrad.defer(dys[1], M, xs[1], N, dw[1], N, M, N, K)
        assert wgrad.defer(dys[2], M, xs[2], N, dw[0], N, M, N, K)  # overlaps record 0
        torch.cuda.synchronize()
        assert float(dw[0].abs().sum()) != 0.0  # records 0 and 1 went out before record 2
    assert not wgrad.defer(dys[0], M, xs[0], N, dw[0], N, M, N, K)  # no scope
    ref = (dys[0].double().t() @ xs[0].double() + dys[2].double().t() @ xs[2].double())
    assert float((dw[0].double() - ref).norm() / ref.norm()) < 2e-6
    ref1 = dys[1].double().t() @ xs[1].double()
    assert float((dw[1].double() - ref1).norm() / ref1.norm()) < 2e-6


def test_losses(cuda):
    from timevqvae.hip.loss import l1_loss, mse_loss
    for f_hip, f_ref in ((mse_loss, F.mse_loss), (l1_loss, F.l1_loss)):
        oc, od, c, d = _run_both(f_hip, f_ref, [(64, 6, 256), (64, 6, 256)], cuda)
        close(od, oc, what="fwd")
        close(d[0].grad, c[0].grad, what="d input")
        close(d[1].grad, c[1].grad, what="d target")


def test_adamw_matches_torch(cuda):
    from timevqvae.hip.optim import FusedAdamW
    gen = torch.Generator().manual_seed(3)
    ps_c = [torch.randn(s, generator=gen).requires_grad_(True) for s in ((64, 32), (7,), (3, 3, 3))]
    ps_d = [p.detach().to(cuda).requires_grad_(True) for p in ps_c]
    oc = torch.optim.AdamW(ps_c, lr=1e-3)
    od = FusedAdamW(ps_d, lr=1e-3)
    for step in range(5):
        grads = [torch.randn(p.shape, generator=gen) for p in ps_c]
        oc.zero_grad()
        od.zero_grad()
        for pc, pd, g in zip(ps_c, ps_d, grads):
            pc.grad = g.clone()
            pd.grad.copy_(g)
        oc.step()
        od.step()
    for pc, pd in zip(ps_c, ps_d):
        torch.testing.assert_close(pd.detach().cpu(), pc.detach(), rtol=1e-6, atol=1e-6)


def test_adamw_skips_gated_parameters_like_torch(cuda):
    """A parameter whose branch did not run (gate 0) is left alone, as torch.optim.AdamW
    leaves a parameter with .grad None: no decay, no moments, no step count."""
    from timevqvae.hip.optim import FusedAdamW

    class Owner:  # stands in for the transformer Encoder (its _touched buffer)
        _touched = torch.ones(2, device=cuda)

    gen = torch.Generator().manual_seed(4)
    shapes = ((5000,), (7, 3), (33,))  # the first spans two chunks
    ps_c = [torch.randn(s, generator=gen).requires_grad_(True) for s in shapes]
    ps_d = [p.detach().to(cuda).requires_grad_(True) for p in ps_c]
    ps_d[0]._tvq_gate = (Owner, 0)
    ps_d[2]._tvq_gate = (Owner, 1)
    oc = torch.optim.AdamW(ps_c, lr=1e-2)
    od = FusedAdamW(ps_d, lr=1e-2)
    pattern = [(1, 1), (0, 1), (0, 0), (1, 0), (1, 1), (0, 1)]
    for step, (k0, k2) in enumerate(pattern):
        grads = [torch.randn(p.shape, generator=gen) for p in ps_c]
        oc.zero_grad(set_to_none=True)
        od.zero_grad()
        Owner._touched.copy_(torch.tensor([float(k0), float(k2)]))
        for i, (pc, pd, g) in enumerate(zip(ps_c, ps_d, grads)):
            used = {0: k0, 1: 1, 2: k2}[i]
            if used:
                pc.grad = g.clone()
                pd.grad.copy_(g)
        oc.step()
        od.step()
    for pc, pd in zip(ps_c, ps_d):
        torch.testing.assert_close(pd.detach().cpu(), pc.detach(), rtol=1e-6, atol=1e-6)


def test_layer_dropout_leaves_skipped_branches_untouched(cuda):
    """x-transformers layer dropout in training (graph-style device decisions): after one
    optimizer step, every parameter of a skipped branch is bitwise unchanged and every
    parameter of a branch that ran has moved."""
    from timevqvae.hip import rng
    from timevqvae.hip.optim import FusedAdamW
    from timevqvae.models.bidirectional_transformer import Encoder
    import contextlib
    import random
    random.seed(3)
    torch.manual_seed(0)
    enc = Encoder(dim=64, depth=4, heads=1, layer_dropout=0.5).to(cuda).train()
    opt = FusedAdamW(enc.parameters(), lr=1e-2)
    x = torch.randn(3, 9, 64, device=cuda)
    for device_decisions in (True, False):
        before = {k: p.detach().clone() for k, p in enc.named_parameters()}
        opt.zero_grad()
        ctx = rng.device_decisions() if device_decisions else contextlib.nullcontext()
        with ctx:
            enc(x).square().sum().backward()
        opt.step()
        touched = enc._touched.cpu().tolist()
        assert 0.0 in touched or device_decisions, touched  # p=0.5 over 8 branches
        for k, p in enc.named_parameters():
            if k.startswith("layers."):
                i = int(k.split(".")[1])
                moved = not torch.equal(p.detach(), before[k])
                assert moved == bool(touched[i]), (k, touched)


@pytest.mark.parametrize("Ci,Co,W", [(16, 16, 32), (64, 64, 8), (8, 8, 64), (128, 16, 32)])
def test_conv_paths_same_dropout_mask(Ci, Co, W, cuda):
    """The dropout mask is a function of (seed, offset, output index) only: the halo
    kernel, the staged GEMM, the split-K GEMM (partials + epilogue) and the default
    per-shape choice drop exactly the same elements."""
    from timevqvae.hip._native import call, ptr, stream_ptr, value
    gen = torch.Generator().manual_seed(3)
    x = torch.randn(5, Ci, 3, W, generator=gen).to(cuda)
    w = torch.randn(Co, Ci, 3, 3, generator=gen).to(cuda) * 0.1
    b = torch.randn(Co, generator=gen).to(cuda)
    r = torch.randn(5, Co, 3, W, generator=gen).to(cuda)
    seed = torch.tensor([1234], dtype=torch.int64, device=cuda)
    nws = value("tvq_conv_workspace", 0, 5, Ci, 3, W, Co, 3, 3, 1, 0)
    ws = torch.empty(nws, device=cuda)
    outs = []
    prev = value("tvq_conv_config", -1)
    try:
        for halo, wsp in ((7, None), (0, None), (0, ws), (3, None)):
            value("tvq_conv_config", halo)
            y = torch.empty(5, Co, 3, W, device=cuda)
            call("tvq_conv2d_fwd", ptr(x), 5, Ci, 3, W, ptr(w), ptr(b), Co, 3, 3, 1, 0, ptr(y),
                 ptr(r), 0.25, ptr(seed), 77, ptr(wsp), stream_ptr())
            outs.append(y)
    finally:
        value("tvq_conv_config", prev)
    torch.cuda.synchronize()
    masks = [o == r for o in outs]
    assert all(torch.equal(masks[0], m) for m in masks[1:])
    torch.testing.assert_close(outs[0], outs[3], rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(outs[0], outs[1], rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(outs[0], outs[2], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("Ci,Co,KH,KW,SW,rep,W", [
    (64, 64, 3, 3, 1, False, 8), (64, 128, 3, 3, 1, False, 8), (128, 128, 3, 3, 1, False, 8),
    (128, 64, 3, 3, 1, False, 8), (64, 128, 1, 1, 1, False, 8), (128, 64, 1, 1, 1, False, 8),
    (32, 64, 3, 4, 2, True, 16), (64, 32, 3, 3, 1, False, 8)])
def test_conv_direct_narrow_maps(Ci, Co, KH, KW, SW, rep, W, cuda):
    """The direct path (conv_d32_kernel) on the LF band's narrow-map shapes (B=64 of the
    (256, C, 3, 8) maps): forward with bias, dropout and residual, and the data / weight
    gradients, against torch fp32 on the CPU; the dropout mask equals the tap kernel's
    (same counter hash at the same output index)."""
    from timevqvae.hip.conv import conv2d
    from timevqvae.hip._native import value
    gen = torch.Generator().manual_seed(Ci * 7 + Co + KW)
    B = 64
    x = torch.randn(B, Ci, 3, W, generator=gen)
    w = torch.randn(Co, Ci, KH, KW, generator=gen) * (Ci * KH * KW) ** -0.5
    bias = torch.randn(Co, generator=gen)
    pad = (0, 0) if rep else (KH // 2, (KW - 1) // 2)
    xc = x.clone().requires_grad_(True)
    wc = w.clone().requires_grad_(True)
    bc = bias.clone().requires_grad_(True)
    xpc = torch.nn.functional.pad(xc, (1, 1, 1, 1), mode="replicate") if rep else xc
    yc = F.conv2d(xpc, wc, bc, stride=(1, SW), padding=pad)
    g = torch.randn(yc.shape, generator=gen)
    res = torch.randn(yc.shape, generator=gen)
    yc.backward(g)
    xd, wd, bd = (t.to(cuda).requires_grad_(True) for t in (x, w, bias))
    yd = conv2d(xd, wd, bd, stride_w=SW, replicate=rep)
    yd.backward(g.to(cuda))
    close(yd, yc, what="fwd")
    close(xd.grad, xc.grad, what="dx")
    close(wd.grad, wc.grad, what="dw")
    close(bd.grad, bc.grad, what="db")
    # dropout + residual epilogue: same mask as the tap kernel (tvq_conv_config 8) at the
    # same (seed, offset)
    from timevqvae.hip._native import call, ptr, stream_ptr
    seed = torch.tensor([4321], dtype=torch.int64, device=cuda)
    nws = value("tvq_conv_workspace", 0, B, Ci, 3, W, Co, KH, KW, SW, int(rep))
    ws = torch.empty(nws, device=cuda)
    xg, wg, bg, rg = x.to(cuda), w.to(cuda), bias.to(cuda), res.to(cuda)
    outs = []
    prev = value("tvq_conv_config", -1)
    try:
        for cfg in (prev, 8):
            value("tvq_conv_config", cfg)
            y = torch.empty(res.shape, device=cuda)
            call("tvq_conv2d_fwd", ptr(xg), B, Ci, 3, W, ptr(wg), ptr(bg), Co, KH, KW, SW, int(rep),
                 ptr(y), ptr(rg), 0.3, ptr(seed), 99, ptr(ws), stream_ptr())
            outs.append(y)
    finally:
        value("tvq_conv_config", prev)
    r0 = res.to(cuda)
    assert torch.equal(outs[0] == r0, outs[1] == r0)
    torch.testing.assert_close(outs[0], outs[1], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("op", ["fwd", "dgrad", "conv1d_fwd", "conv1d_dgrad", "fwd64", "dgrad64",
                                "fwd128n", "dgrad128n"])
def test_conv_wide_tile_matches_tap(op, cuda):
    """The 32x32-MFMA wide-channel tile (C, N >= 128 on a full grid) computes each output as
    the same k-ordered fma chain as the tap-major kernel's unsplit path: bitwise equal to it,
    and within the fp32 tolerance of torch's CPU conv."""
    from timevqvae.hip._native import call, ptr, stream_ptr, value
    gen = torch.Generator().manual_seed(11)
    if op.startswith("conv1d"):
        B, Ci, Co, H, W, KH, KW = 256, 128, 256, 1, 96, 1, 3
    elif op.endswith("64"):  # LF band 64-channel ResBlock conv: the 64-channel tile
        B, Ci, Co, H, W, KH, KW = 256, 64, 64, 3, 8, 3, 3
    elif op.endswith("128n"):  # 128 channels on a narrow map: 64-channel tile, 2 column tiles
        B, Ci, Co, H, W, KH, KW = 256, 128, 128, 3, 8, 3, 3
    else:
        B, Ci, Co, H, W, KH, KW = 192, 128, 128, 3, 32, 3, 3
    x = torch.randn(B, Ci, H, W, generator=gen)
    w = torch.randn(Co, Ci, KH, KW, generator=gen) * 0.05
    bias = torch.randn(Co, generator=gen)
    dy = torch.randn(B, Co, H, W, generator=gen)
    xd, wd, bd, dyd = x.to(cuda), w.to(cuda), bias.to(cuda), dy.to(cuda)
    outs = []
    prev = value("tvq_conv_config", -1)
    try:
        # wide tile (packed) at K-stage depth BK = 64, 32, 16, with 12 and 4 waves per block
        # | tap, unsplit, raw
        # (128: the 64-channel variant, which is what the narrow "64"/"128n" maps exercise;
        # without it those maps run the split-K tap kernel, a different summation order)
        cfgs = ((0, True), (16, True), (32, True), (64, True), (80, True), (8, False))
        if op.endswith(("64", "128n")):
            cfgs = ((128, True), (8, False))
        for cfg, use_ws in cfgs:
            value("tvq_conv_config", cfg)
            if "fwd" in op:
                y = torch.empty(B, Co, H, W, device=cuda)
                ws = torch.empty(value("tvq_conv_workspace", 0, B, Ci, H, W, Co, KH, KW, 1, 0),
                                 device=cuda) if use_ws else None
                call("tvq_conv2d_fwd", ptr(xd), B, Ci, H, W, ptr(wd), ptr(bd), Co, KH, KW, 1, 0,
                     ptr(y), None, 0.0, None, 0, ptr(ws), stream_ptr())
            else:
                y = torch.empty(B, Ci, H, W, device=cuda)
                ws = torch.empty(value("tvq_conv_workspace", 2, B, Ci, H, W, Co, KH, KW, 1, 0),
                                 device=cuda) if use_ws else None
                call("tvq_conv2d_dgrad", ptr(dyd), B, Co, H, W, ptr(wd), Ci, KH, KW, 1, 0, ptr(y),
                     W, ptr(ws), stream_ptr())
            outs.append(y)
    finally:
        value("tvq_conv_config", prev)
    torch.cuda.synchronize()
    for o in outs[:-1]:
        assert torch.equal(o, outs[-1])
    pad = (KH // 2, (KW - 1) // 2)
    if "fwd" in op:
        ref = F.conv2d(x, w, bias, padding=pad)
    else:
        ref = torch.nn.grad.conv2d_input(x.shape, w, dy, padding=pad)
    close(outs[0].cpu(), ref, what=op)


@pytest.mark.gpu
@pytest.mark.parametrize("B,Ci,Co", [(256, 64, 64), (256, 128, 64), (48, 64, 128), (40, 64, 64)])
def test_conv_wgrad_narrow_image_batched(B, Ci, Co, cuda):
    """conv_wgrad_w8_kernel (3x3 on (B, C, 3, 8) maps, 16 images per block, the 4 waves'
    partial tiles summed in order) against torch fp32 on the CPU at the step's batch; B = 40
    (not a multiple of 16) takes the halo kernel instead."""
    from timevqvae.hip.conv import conv2d
    gen = torch.Generator().manual_seed(B + Ci + Co)
    x = torch.randn(B, Ci, 3, 8, generator=gen)
    w = torch.randn(Co, Ci, 3, 3, generator=gen) * (Ci * 9) ** -0.5
    b = torch.randn(Co, generator=gen)
    g = torch.randn(B, Co, 3, 8, generator=gen)
    wc, bc = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    F.conv2d(x, wc, bc, padding=(1, 1)).backward(g)
    wd, bd = w.to(cuda).requires_grad_(True), b.to(cuda).requires_grad_(True)
    conv2d(x.to(cuda), wd, bd).backward(g.to(cuda))
    close(wd.grad, wc.grad, what="dw")
    close(bd.grad, bc.grad, what="db")


@pytest.mark.parametrize("B,Lin,D,Lout", [(4, 32, 128, 96), (3, 25, 70, 97), (2, 130, 16, 300)])
def test_upsample_nearest_t(B, Lin, D, Lout, cuda):
    """(b, n, d) -> F.interpolate(x.transpose(1, 2), Lout, 'nearest'): forward and the
    gradient (tiled kernel for Lin <= 128, the per-element one above) against torch."""
    from timevqvae.hip.xf import upsample_nearest_t
    gen = torch.Generator().manual_seed(5)
    x = torch.randn(B, Lin, D, generator=gen)
    gy = torch.randn(B, D, Lout, generator=gen)
    xc = x.clone().requires_grad_(True)
    yc = F.interpolate(xc.transpose(1, 2), Lout, mode="nearest")
    yc.backward(gy)
    xd = x.to(cuda).requires_grad_(True)
    yd = upsample_nearest_t(xd, Lout)
    yd.backward(gy.to(cuda))
    torch.cuda.synchronize()
    assert torch.equal(yd.cpu(), yc.detach())
    close(xd.grad, xc.grad, what="dx")



@pytest.mark.parametrize("zero_after", [False, True])
def test_adamw_step_pair_equals_two_steps(zero_after, cuda):
    """hip.optim.step_pair (tvq_adamw2: both optimizers' step counts, then both updates, two
    launches) gives the same bits as two FusedAdamW.step calls, with different
    hyper-parameters per optimizer; with zero_after_step the gradients read are zeroed and the
    next zero_grad launches nothing."""
    from timevqvae.hip.optim import FusedAdamW, step_pair
    gen = torch.Generator().manual_seed(4)

    def make():
        torch.manual_seed(0)
        m1 = torch.nn.Sequential(torch.nn.Linear(37, 19), torch.nn.Linear(19, 5)).to(cuda)
        m2 = torch.nn.Linear(300, 77).to(cuda)
        o1 = FusedAdamW(m1.parameters(), lr=1e-3, weight_decay=0.01)
        o2 = FusedAdamW(m2.parameters(), lr=3e-4, betas=(0.8, 0.95), eps=1e-6, weight_decay=0.1)
        o1.zero_after_step = o2.zero_after_step = zero_after
        return o1, o2

    ref, got = make(), make()
    for _ in range(3):
        g1 = torch.randn(ref[0].numel, generator=gen).to(cuda)
        g2 = torch.randn(ref[1].numel, generator=gen).to(cuda)
        for (o1, o2) in (ref, got):
            o1.zero_grad()
            o2.zero_grad()
            o1.flat_grad += g1
            o2.flat_grad += g2
        ref[0].step()
        ref[1].step()
        step_pair(*got)
        for a, b in zip(ref, got):
            assert torch.equal(a.flat, b.flat) and torch.equal(a.exp_avg, b.exp_avg)
            assert torch.equal(a.exp_avg_sq, b.exp_avg_sq) and torch.equal(a.seg_step, b.seg_step)
            assert torch.equal(a.flat_grad, b.flat_grad)
            assert bool((b.flat_grad == 0).all()) == zero_after


def test_adamw_zero_after_step_clears_gated_segments(cuda):
    """zero_after_step with a gated-off segment (layer dropout skipped the branch): the
    segment's parameters and moments are untouched, and its gradient -- here a NaN a dropped
    branch could leave -- is still cleared, so it cannot be applied when the gate reopens."""
    from timevqvae.hip.optim import FusedAdamW, step_pair
    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(300, 20), torch.nn.Linear(20, 7)).to(cuda)
    o = FusedAdamW(m.parameters(), lr=1e-3, weight_decay=0.01)
    o2 = FusedAdamW(torch.nn.Linear(5, 3).to(cuda).parameters(), lr=1e-3)
    o.zero_after_step = o2.zero_after_step = True
    o.zero_grad()
    o2.zero_grad()
    o.flat_grad.normal_()
    o.flat_grad[:6000] = float("nan")  # the first segment: Linear(300, 20).weight
    before = o.flat.clone()
    o.gates.fill_(1.0)
    o.gates[0] = 0.0
    o2.gates.fill_(1.0)
    step_pair(o, o2, gates_ready=True)
    torch.cuda.synchronize()
    assert bool((o.flat_grad == 0).all())
    assert torch.equal(o.flat[:6000], before[:6000])
    assert bool((o.exp_avg[:6000] == 0).all()) and float(o.seg_step[0]) == 0.0
    assert bool(torch.isfinite(o.flat).all()) and not torch.equal(o.flat[6000:], before[6000:])
    o.gates.fill_(1.0)  # the gate reopens: the update sees a zero gradient, not the NaN
    o.zero_grad()
    o.step(gates_ready=True)
    assert bool(torch.isfinite(o.flat).all())


@pytest.mark.parametrize("D", [32, 64, 128, 256, 48])
@pytest.mark.parametrize("M", [1, 7, 1000, 99328])
def test_norm_fwd_narrow_rows_vs_torch(D, M):
    """RMSNorm / LayerNorm forward on the narrow-row vector kernels (D = 4L, 64/L rows per
    wave; D = 48 takes the one-wave-per-row form) against torch fp32, ragged row counts
    (tolerance: fp32 sums in another order, rel 1e-5 of the output scale)."""
    from timevqvae.hip._native import plan_trace
    from timevqvae.hip.xf import layer_norm, rmsnorm
    torch.manual_seed(D + M)
    x = torch.randn(M, D, device="cuda") * 3 + 0.5
    g = torch.rand(D, device="cuda") + 0.5
    b = torch.randn(D, device="cuda")
    with torch.no_grad(), plan_trace() as tr:
        y = rmsnorm(x, g)
        z = layer_norm(x, g, b, 1e-5)
    vec = D in (32, 64, 128, 256)
    assert any(t.startswith(f"rmsnorm_fwd_vec D{D}") for t in tr.lines) == vec
    assert any(t.startswith(f"layernorm_fwd_vec D{D}") for t in tr.lines) == vec
    ref_y = x / x.norm(dim=-1, keepdim=True).clamp_min(1e-12) * D ** 0.5 * g
    ref_z = F.layer_norm(x, (D,), g, b, 1e-5)
    assert (y - ref_y).abs().max().item() <= 1e-5 * ref_y.abs().max().item()
    assert (z - ref_z).abs().max().item() <= 1e-5 * ref_z.abs().max().item()
