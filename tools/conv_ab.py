"""Time one conv (fwd and dgrad) under two tvq_conv_config settings, weights from a pack
cache scope (as in the step).  usage: python tools/conv_ab.py B Ci Co H W cfgA cfgB"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "t-vq-vae-trajgen_amd"))
import torch  # noqa: E402

from timevqvae.hip._native import value  # noqa: E402
from timevqvae.hip.conv import PackCache, conv2d  # noqa: E402


def main():
    B, Ci, Co, H, W, ca, cb = [int(v) for v in sys.argv[1:8]]
    dev = torch.device("cuda", 0)
    x = torch.randn(B, Ci, H, W, device=dev, requires_grad=True)
    w = torch.randn(Co, Ci, 3, 3, device=dev) * 0.05
    w.requires_grad_(True)
    b = torch.zeros(Co, device=dev)
    for cfg in (ca, cb, ca, cb):
        value("tvq_conv_config", cfg)
        pc = PackCache(dev, 1 << 20)
        with pc.scope():
            y = conv2d(x, w, b)
            g = torch.randn_like(y)
            y.backward(g)
        with pc.scope():
            for _ in range(3):
                conv2d(x, w, b)
            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            e[0].record()
            for _ in range(20):
                conv2d(x, w, b)
            e[1].record()
            for _ in range(20):
                y = conv2d(x, w, b)
                torch.autograd.grad(y, x, g)
            e[2].record()
            torch.cuda.synchronize()
        f = e[0].elapsed_time(e[1]) / 20 * 1e3
        fb = e[1].elapsed_time(e[2]) / 20 * 1e3
        print(f"cfg {cfg}: fwd {f:.1f} us, fwd+dgrad {fb:.1f} us")


if __name__ == "__main__":
    main()
