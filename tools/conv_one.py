"""Run one conv op of tools/conv_shapes_bench.SHAPES `reps` times (for rocprofv3 PMC passes).
usage: python tools/conv_one.py <shape index> <fwd|dgrad|wgrad> [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "t-vq-vae-trajgen_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from conv_shapes_bench import B, SHAPES  # noqa: E402
from timevqvae.hip._native import call, ptr, stream_ptr, value  # noqa: E402


def main():
    si, op = int(sys.argv[1]), sys.argv[2]
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    n, Ci, Co, H, Wi, KH, KW, SW, rep, tr = SHAPES[si]
    assert not tr
    dev = torch.device("cuda", 0)
    Wo = value("tvq_conv_out_width", Wi, KW, SW, 0)
    x = torch.randn(B, Ci, H, Wi, device=dev)
    w = torch.randn(Co, Ci, KH, KW, device=dev) * 0.05
    b = torch.zeros(Co, device=dev)
    y = torch.empty(B, Co, H, Wo, device=dev)
    dy = torch.randn_like(y)
    dx = torch.empty_like(x)
    dw = torch.empty_like(w)
    db = torch.empty_like(b)
    opi = {"fwd": 0, "dgrad": 2, "wgrad": 4}[op]
    ws = torch.empty(value("tvq_conv_workspace", opi, B, Ci, H, Wi, Co, KH, KW, SW, rep), device=dev)
    for _ in range(reps):
        if op == "fwd":
            call("tvq_conv2d_fwd", ptr(x), B, Ci, H, Wi, ptr(w), ptr(b), Co, KH, KW, SW, rep, ptr(y),
                 None, 0.0, None, 0, ptr(ws), stream_ptr())
        elif op == "dgrad":
            call("tvq_conv2d_dgrad", ptr(dy), B, Co, H, Wo, ptr(w), Ci, KH, KW, SW, rep, ptr(dx), Wi,
                 ptr(ws), stream_ptr())
        else:
            call("tvq_conv2d_wgrad", ptr(x), B, Ci, H, Wi, ptr(dy), Co, Wo, KH, KW, SW, rep, ptr(dw),
                 ptr(db), 0, ptr(ws), stream_ptr())
    torch.cuda.synchronize()
    print("ok", SHAPES[si], op)


if __name__ == "__main__":
    main()
