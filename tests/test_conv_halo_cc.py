"""The channel-chunked halo conv (csrc/tvq_conv.hip conv_halo_cc_kernel): wide input into
<= 16 outputs at stride 1 -- the HF decoder ResBlock's 128 -> 16 3x3 conv and 1x1
projection (vq_vae.py:13-62) and the data gradients of the 16 -> 128 convs -- against torch
fp32 (F.conv2d, autograd), at the benched B = 256 and the sampler's B = 1024 (forward),
and checked to dispatch the kernel.  The kernel is opt-in (tvq_conv_config bit 2048: it
measured slower than the tap GEMM in the step); the tests switch it on and restore the
setting.  Tolerance rel-L2 1e-5 (fp32, MFMA summation order)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture
def hcc_on():
    from timevqvae.hip._native import lib
    prev = lib().tvq_conv_config(-1)
    lib().tvq_conv_config(prev | 2048)
    yield
    lib().tvq_conv_config(prev)


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).norm() / (b.norm() + 1e-30))


@pytest.mark.parametrize("B,Ci,Co,W,k", [(256, 128, 16, 32, 3), (256, 128, 16, 32, 1),
                                         (1024, 128, 16, 32, 3), (5, 64, 12, 17, 3),
                                         (3, 96, 16, 8, 1)])
def test_halo_cc_forward(B, Ci, Co, W, k, cuda, hcc_on):
    from timevqvae.hip._native import plan_trace
    from timevqvae.hip.conv import conv2d
    torch.manual_seed(B + Ci + Co + W + k)
    x = torch.randn(B, Ci, 3, W, device=cuda)
    w = torch.randn(Co, Ci, k, k, device=cuda) * (Ci * k * k) ** -0.5
    b = torch.randn(Co, device=cuda) * 0.1
    with torch.no_grad(), plan_trace() as tr:
        y = conv2d(x, w, b)
        torch.cuda.synchronize()
    assert tr.has("conv_halo_cc"), tr.lines
    want = F.conv2d(x, w, b, padding=k // 2)
    assert rel(y, want) < 1e-5, rel(y, want)


@pytest.mark.parametrize("k", [3, 1])
def test_halo_cc_data_gradient(k, cuda, hcc_on):
    """dx of the HF encoder's 16 -> 128 conv (B = 256, W = 32): the 128 -> 16 gather."""
    from timevqvae.hip._native import plan_trace
    from timevqvae.hip.conv import conv2d
    torch.manual_seed(k)
    x = torch.randn(256, 16, 3, 32, device=cuda, requires_grad=True)
    w = (torch.randn(128, 16, k, k, device=cuda) * (16 * k * k) ** -0.5).requires_grad_(False)
    b = torch.randn(128, device=cuda) * 0.1
    gy = torch.randn(256, 128, 3, 32, device=cuda)
    with plan_trace() as tr:
        y = conv2d(x, w, b)
        (dx,) = torch.autograd.grad(y, x, gy)
        torch.cuda.synchronize()
    assert tr.has("conv_halo_cc"), tr.lines
    xr = x.detach().clone().requires_grad_(True)
    (want,) = torch.autograd.grad(F.conv2d(xr, w, b, padding=k // 2), xr, gy)
    assert rel(dx, want) < 1e-5, rel(dx, want)
