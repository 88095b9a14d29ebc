"""Fused small-channel ResBlock vs the per-op path at the step's shapes (B=256): graph-
replayed device time of the training forward, forward+backward and the eval forward.
usage: python tools/resblock_bench.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "t-vq-vae-trajgen_amd"))
import torch  # noqa: E402


def gtime(fn, reps=20):
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=st):
            for _ in range(reps):
                fn()
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(3):
            g.replay()
        e1.record(st)
        torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (3 * reps)


def main():
    from timevqvae.hip import resblock
    from timevqvae.models.vq_vae import ResBlock
    dev = torch.device("cuda", 0)
    for C, W in ((8, 64), (16, 32), (32, 16), (64, 8)):
        m = ResBlock(C, C, False, dropout=0.3).to(dev)
        x = torch.randn(256, C, 3, W, device=dev, requires_grad=True)
        gy = torch.randn(256, C, 3, W, device=dev)
        row = []
        for fused in (False, True):
            resblock.ENABLED = fused
            if fused and not resblock.supported(x, C, C):
                row.append("   n/a")
                continue
            m.train()
            with torch.no_grad():
                tf = gtime(lambda: m(x))

            def fb():
                y = m(x)
                torch.autograd.backward(y, gy, inputs=[x] + list(m.parameters()))
            tb = gtime(fb, reps=5)
            m.eval()
            with torch.no_grad():
                te = gtime(lambda: m(x))
            row.append(f"fwd {tf:6.1f} fwd+bwd {tb:6.1f} eval {te:6.1f}")
        print(f"C={C:3d} W={W:3d}  per-op: {row[0]} | fused: {row[1]}", flush=True)


if __name__ == "__main__":
    main()
