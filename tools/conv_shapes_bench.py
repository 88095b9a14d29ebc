"""Per-shape timing of the conv engine at the joint step's shapes (config B).

For every conv of the step: fwd, dgrad and wgrad times (HIP events, 20 reps) against the
max(MFMA, HBM) floor.  usage: python tools/conv_shapes_bench.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "t-vq-vae-trajgen_amd"))
import torch  # noqa: E402

from timevqvae.hip._native import call, ptr, stream_ptr, value  # noqa: E402

# (count per step, Ci, Co, Hin, Win, KH, KW, SW, replicate, transposed)
SHAPES = [
    (4, 4, 8, 3, 128, 3, 4, 2, 1, 0), (24, 8, 8, 3, 64, 3, 3, 1, 0, 0),
    (4, 8, 16, 3, 64, 3, 4, 2, 1, 0), (4, 12, 4, 3, 257, 3, 4, 2, 1, 0),
    (25, 16, 16, 3, 32, 3, 3, 1, 0, 0), (2, 16, 32, 3, 32, 3, 4, 2, 1, 0),
    (2, 16, 128, 3, 32, 1, 1, 1, 0, 0), (2, 16, 128, 3, 32, 3, 3, 1, 0, 0),
    (12, 32, 32, 3, 16, 3, 3, 1, 0, 0), (2, 32, 64, 3, 16, 3, 4, 2, 1, 0),
    (13, 64, 64, 3, 8, 3, 3, 1, 0, 0), (2, 64, 128, 3, 8, 1, 1, 1, 0, 0),
    (2, 64, 128, 3, 8, 3, 3, 1, 0, 0), (1, 128, 16, 3, 32, 1, 1, 1, 0, 0),
    (1, 128, 16, 3, 32, 3, 3, 1, 0, 0), (1, 128, 64, 3, 8, 1, 1, 1, 0, 0),
    (1, 128, 64, 3, 8, 3, 3, 1, 0, 0), (2, 128, 128, 3, 8, 3, 3, 1, 0, 0),
    (2, 128, 128, 3, 32, 3, 3, 1, 0, 0),
    (2, 4, 12, 3, 128, 3, 4, 2, 0, 1), (2, 8, 4, 3, 64, 3, 4, 2, 0, 1),
    (2, 12, 12, 3, 256, 3, 4, 2, 0, 1), (2, 16, 8, 3, 32, 3, 4, 2, 0, 1),
    (1, 32, 16, 3, 16, 3, 4, 2, 0, 1), (1, 64, 32, 3, 8, 3, 4, 2, 0, 1),
    (1, 128, 256, 1, 96, 1, 3, 1, 0, 0), (1, 256, 128, 1, 96, 1, 3, 1, 0, 0),
]
B = 256


def timeit(fn, reps=20):
    """GPU time per call: `reps` calls captured in one HIP graph (no host launch cost)."""
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        for _ in range(3):
            fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    cur = torch.cuda.current_stream()
    e0.record(cur)
    g.replay()
    e1.record(cur)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3  # us


def main():
    only = {int(a) for a in sys.argv[1].split(",")} if len(sys.argv) > 1 else None
    dev = torch.device("cuda", 0)
    if "TVQ_CONV_HALO" in os.environ:  # tvq_conv_config bits (1/2 halo, 256: no small direct)
        value("tvq_conv_config", int(os.environ["TVQ_CONV_HALO"]))
    tot = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0, "floor": 0.0}
    print(f"{'n':>3} {'Ci':>4} {'Co':>4} {'W':>4} k    {'fwd':>7} {'dgrad':>7} {'wgrad':>7}  floor(us)")
    for si, (n, Ci, Co, H, Wi, KH, KW, SW, rep, tr) in enumerate(SHAPES):
        if only is not None and si not in only:
            continue
        Wo = value("tvq_conv_out_width", Wi, KW, SW, tr)
        x = torch.randn(B, Ci, H, Wi, device=dev)
        w = torch.randn(*((Ci, Co) if tr else (Co, Ci)), KH, KW, device=dev) * 0.05
        b = torch.zeros(Co, device=dev)
        y = torch.empty(B, Co, H, Wo, device=dev)
        dy = torch.randn_like(y)
        dx = torch.empty_like(x)
        dw = torch.empty_like(w)
        db = torch.empty_like(b)
        def ws(op):
            return torch.empty(value("tvq_conv_workspace", op, B, Ci, H, Wi, Co, KH, KW, SW, rep),
                               device=dev)
        if not tr:
            wf, wd, wg = ws(0), ws(2), ws(4)
            f = lambda: call("tvq_conv2d_fwd", ptr(x), B, Ci, H, Wi, ptr(w), ptr(b), Co, KH, KW, SW,  # noqa
                             rep, ptr(y), None, 0.0, None, 0, ptr(wf), stream_ptr())
            d = lambda: call("tvq_conv2d_dgrad", ptr(dy), B, Co, H, Wo, ptr(w), Ci, KH, KW, SW, rep,  # noqa
                             ptr(dx), Wi, ptr(wd), stream_ptr())
            g = lambda: call("tvq_conv2d_wgrad", ptr(x), B, Ci, H, Wi, ptr(dy), Co, Wo, KH, KW, SW,  # noqa
                             rep, ptr(dw), ptr(db), 0, ptr(wg), stream_ptr())
        else:
            wf, wd, wg = ws(1), ws(3), ws(5)
            f = lambda: call("tvq_convT2d_fwd", ptr(x), B, Ci, H, Wi, ptr(w), ptr(b), Co, KH, KW, SW,  # noqa
                             ptr(y), None, ptr(wf), stream_ptr())
            d = lambda: call("tvq_convT2d_dgrad", ptr(dy), B, Co, H, Wo, ptr(w), Ci, KH, KW, SW,  # noqa
                             ptr(dx), Wi, ptr(wd), stream_ptr())
            g = lambda: call("tvq_convT2d_wgrad", ptr(x), B, Ci, H, Wi, ptr(dy), Co, Wo, KH, KW, SW,  # noqa
                             ptr(dw), 0, ptr(wg), stream_ptr())
        tf, td, tg = timeit(f), timeit(d), timeit(g)
        flops = 2.0 * B * H * (Wo if not tr else Wi) * Co * Ci * KH * KW
        byts = 4.0 * (x.numel() + y.numel())
        floor = max(flops / 157.3e12, byts / 8e12) * 1e6
        for k, v in (("fwd", tf), ("dgrad", td), ("wgrad", tg), ("floor", 3 * floor)):
            tot[k] += n * v
        print(f"{n:3d} {Ci:4d} {Co:4d} {Wo:4d} {KH}x{KW}{'T' if tr else ' '} {tf:7.1f} {td:7.1f} {tg:7.1f}  "
              f"{floor:6.1f}")
    print("per-step totals (us): " + ", ".join(f"{k} {v:.0f}" for k, v in tot.items()))


if __name__ == "__main__":
    main()
