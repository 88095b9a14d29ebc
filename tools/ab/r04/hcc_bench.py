"""A/B of the channel-chunked halo conv (tvq_conv_config bit 2048) against the default
dispatch on the wide-input -> 16-output shapes of the step and the sampler."""
import sys

import torch

sys.path.insert(0, "t-vq-vae-trajgen_amd")
from timevqvae.hip._native import lib  # noqa: E402
from timevqvae.hip.conv import conv2d  # noqa: E402


def t_us(fn, reps=50):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


dev = torch.device("cuda:0")
prev = lib().tvq_conv_config(-1)
for B, k in [(256, 3), (256, 1), (1024, 3), (1024, 1)]:
    x = torch.randn(B, 128, 3, 32, device=dev)
    w = torch.randn(16, 128, k, k, device=dev) * 0.05
    b = torch.randn(16, device=dev)
    res = {}
    for name, cfg in (("tap", prev), ("hcc", prev | 2048)):
        lib().tvq_conv_config(cfg)
        with torch.no_grad():
            res[name] = t_us(lambda: conv2d(x, w, b))
    lib().tvq_conv_config(prev)
    print(f"B={B} k={k}: tap {res['tap']:.1f} us  halo_cc {res['hcc']:.1f} us", flush=True)
