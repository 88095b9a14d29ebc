"""Upscale's first conv on the LF token grid (hip.upscale, csrc/tvq_upscale.hip) against
torch fp32 / fp64 references of the reference's own expression
(bidirectional_transformer.py:12-30: interpolate(nearest) -> Conv1d(k3, pad 1) -> GELU
[-> BatchNorm1d]).  The token-grid form reassociates the conv's sums (A + B + C per token
instead of the 3d-term dot product), so the bars are fp32 relative tolerances, written per
test."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

SHAPES = [  # (B, n, d, H, f)
    (256, 24, 128, 256, 4),  # the HF prior of configs[2]: 24 LF tokens -> 96 HF positions
    (3, 5, 16, 70, 2),       # H not a multiple of the 64-channel block, f = 2
    (2, 7, 32, 33, 3),       # odd f
    (4, 1, 8, 5, 6),         # one token: both ends are padding
    (1, 60, 64, 130, 4),     # m = 240, the largest supported
]


def _ref(x, w, b, m):
    return F.gelu(F.conv1d(F.interpolate(x.transpose(1, 2), size=m, mode="nearest"), w, b,
                           padding=1))


@pytest.mark.parametrize("B,n,d,H,f", SHAPES)
def test_upsample_conv_gelu_fwd_bwd_vs_torch(B, n, d, H, f, cuda):
    from timevqvae.hip.upscale import supported, upsample_conv_gelu
    torch.manual_seed(B * 1000 + n)
    m = f * n
    x = torch.randn(B, n, d, dtype=torch.float64)
    w = torch.randn(H, d, 3, dtype=torch.float64) / (3 * d) ** 0.5
    b = torch.randn(H, dtype=torch.float64) * 0.1
    gy = torch.randn(B, H, m, dtype=torch.float64)
    xr, wr, br = (t.clone().requires_grad_(True) for t in (x, w, b))
    ref = _ref(xr, wr, br, m)
    ref.backward(gy)
    xg, wg, bg = (t.float().to(cuda).requires_grad_(True) for t in (x, w, b))
    assert supported(xg, m, wg)
    y = upsample_conv_gelu(xg, m, wg, bg)
    y.backward(gy.float().to(cuda))
    torch.cuda.synchronize()

    def rel(a, r):
        return float((a.detach().cpu().double() - r).abs().max() / r.abs().max())
    # fp32 sums of <= 3 d products against the fp64 reference
    assert rel(y, ref.detach()) < 2e-6
    assert rel(xg.grad, xr.grad) < 5e-6
    assert rel(wg.grad, wr.grad) < 5e-6
    assert rel(bg.grad, br.grad) < 5e-6


def test_upscale_module_token_grid_equals_upsample_path(cuda):
    """The Upscale module (train-mode BatchNorm) on the token grid against its upsample ->
    conv path: outputs, input gradient, every parameter gradient and the BN running
    statistics within 1e-5 relative (configs[2] shape)."""
    import copy

    from timevqvae.models import bidirectional_transformer as bt
    torch.manual_seed(0)
    up = bt.Upscale(128, 128, 256).to(cuda).train()
    up2 = copy.deepcopy(up)
    x = torch.randn(256, 24, 128, device=cuda)
    gy = torch.randn(256, 96, 128, device=cuda)
    outs = []
    for mod, on in ((up, True), (up2, False)):
        bt.UPS_ON_TOKENS = on
        try:
            xi = x.clone().requires_grad_(True)
            y = mod(xi, 96)
            y.backward(gy)
        finally:
            bt.UPS_ON_TOKENS = True
        outs.append((y.detach(), xi.grad, {k: p.grad for k, p in mod.named_parameters()},
                     {k: v.clone() for k, v in mod.state_dict().items()}))
    (y1, g1, p1, s1), (y2, g2, p2, s2) = outs

    def rel(a, r):
        return float((a - r).abs().max() / r.abs().max().clamp_min(1e-30))
    assert rel(y1, y2) < 1e-5
    assert rel(g1, g2) < 1e-5
    for k in p1:
        assert rel(p1[k], p2[k]) < 1e-5, k
    for k in s1:
        if s1[k].is_floating_point():
            assert rel(s1[k], s2[k]) < 1e-5, k


def test_upsample_conv_gelu_bn_eval_vs_torch(cuda):
    """The sampling form: BatchNorm1d_eval(GELU(conv)) in the combine launch against torch
    (1024 sequences as in configs[4]; the epilogue's GELU is the A&S erf form, <= 1.5e-7
    absolute)."""
    from timevqvae.hip.upscale import upsample_conv_gelu_bn_eval
    torch.manual_seed(1)
    B, n, d, H, m = 1024, 24, 128, 256, 96
    x = torch.randn(B, n, d, device=cuda)
    w = torch.randn(H, d, 3, device=cuda) / (3 * d) ** 0.5
    b = torch.randn(H, device=cuda) * 0.1
    bn = torch.nn.BatchNorm1d(H).to(cuda).eval()
    with torch.no_grad():
        bn.running_mean.normal_()
        bn.running_var.uniform_(0.5, 2.0)
        bn.weight.normal_()
        bn.bias.normal_()
        y = upsample_conv_gelu_bn_eval(x, m, w, b, bn)
        ref = bn(F.gelu(F.conv1d(F.interpolate(x.double().transpose(1, 2), size=m), w.double(),
                                 b.double(), padding=1)).float())
    torch.cuda.synchronize()
    assert float((y - ref).abs().max() / ref.abs().max()) < 5e-6


def test_hf_prior_takes_token_grid(cuda):
    """The HF prior's training forward and its sampling head both take the token-grid conv
    (plan trace), not the upsample -> conv path."""
    from timevqvae.hip._native import plan_trace
    from timevqvae.models import BidirectionalTransformer
    tf = BidirectionalTransformer("hf", 96, {"lf": 64, "hf": 64}, 128, hidden_dim=32, n_layers=1,
                                  heads=1, ff_mult=1, use_rmsnorm=True, p_unconditional=0.2,
                                  n_classes=5, num_tokens_l=24).to(cuda).train()
    sl = torch.randint(0, 65, (8, 24), device=cuda)
    sh = torch.randint(0, 65, (8, 96), device=cuda)
    with plan_trace() as tr:
        tf(sl, sh).sum().backward()
    assert any(t.startswith("ups_combine B8 n24 f4 H256 mode0") for t in tr.lines), tr.lines
    assert any(t.startswith("ups_sums B8 n24 f4 H256") for t in tr.lines)
    tf.eval()
    with torch.no_grad(), plan_trace() as tr:
        tf._head_hf_eval(sl, sh, None)
    assert any(t.startswith("ups_combine B8 n24 f4 H256 mode2") for t in tr.lines), tr.lines
