"""Time the VQ kernels at config-B token counts (HF 24576 x 512 x 128, LF 6144)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "t-vq-vae-trajgen_amd"))
import torch
from timevqvae.models import VectorQuantize

dev = torch.device("cuda:0")
for name, W in (("LF", 8), ("HF", 32)):
    z = torch.randn(256, 128, 3, W, device=dev)
    x = z.flatten(2).transpose(1, 2)
    vq = VectorQuantize(128, 512).to(dev)
    for mode in ("eval", "train"):
        vq.train(mode == "train")
        for _ in range(3):
            vq(x)
        torch.cuda.synchronize()
        n = 50
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            vq(x)
        e1.record(); torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / n
        M = x.shape[0] * x.shape[1]
        print(f"{name} {mode}: M={M} {ms*1e3:.1f} us/call  ({2*M*512*128/ms/1e9:.1f} TFLOP/s dist)")
