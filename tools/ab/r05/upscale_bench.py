"""Time the HF prior's Upscale conv1 (Conv1d 128 -> 256, k3 on 96 positions) at the
sampler's batch (1024) and the training batch (256): the eval-fused post variant
(conv + GELU + BN eval) against the plain conv."""
import sys

import torch

sys.path.insert(0, "t-vq-vae-trajgen_amd")
from timevqvae.hip.conv import conv2d, conv2d_bn_eval  # noqa: E402
from timevqvae.models.bidirectional_transformer import Upscale  # noqa: E402


def t(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1000


from timevqvae.hip._native import lib  # noqa: E402

torch.manual_seed(0)
up = Upscale(128, 128, 256).cuda().eval()
BITS = int(sys.argv[1]) if len(sys.argv) > 1 else 0  # tvq_conv_config bits to add (16: BK 32)
if BITS:
    cur = lib().tvq_conv_config(-1)
    lib().tvq_conv_config(cur | BITS)
    print("conv config", cur, "->", cur | BITS)
c = up.conv
for B in (256, 1024):
    x = torch.randn(B, 128, 96, device="cuda")
    with torch.no_grad():
        us_post = t(lambda: conv2d_bn_eval(x, c[0].weight, c[0].bias, c[2], None, pre_gelu=True))
        us_plain = t(lambda: conv2d(x, c[0].weight, c[0].bias))
        xs = torch.randn(B, 24, 128, device="cuda")
        us_all = t(lambda: up(xs, 96))
    fl = 2 * B * 96 * 384 * 256
    print(f"B={B} post {us_post:.1f} us ({fl / us_post / 1e6:.1f} TF/s)  plain {us_plain:.1f} us "
          f"({fl / us_plain / 1e6:.1f} TF/s)  upscale {us_all:.1f} us", flush=True)
