"""Per-block phase timestamps of the fused ResBlock kernels (timing build:
lib_ab/libtvq_hip_rbtime.so, tvq_resblock.hip compiled with -DRB_TIMING).
Marks (bwd1 / bwd2): m0 start, m1 loads issued + borders + panel stored, m2 inputs staged
(barrier), m3 weight-gradient items done, m4 conv items done (barrier), m5 epilogue stored,
m6 channel partials published, m7 last-block finish.  fwd1: m0 start, m1 panel stored,
m2 staged, m3 conv done, m4 epilogue, m5 partials, m6 finish.
usage: python tools/rb_timing.py"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["TVQ_HIP_LIB"] = os.path.join(ROOT, "t-vq-vae-trajgen_amd", "lib_ab", "libtvq_hip_rbtime.so")
sys.path.insert(0, os.path.join(ROOT, "t-vq-vae-trajgen_amd"))
import torch  # noqa: E402

KINDS = ["fwd1", "fwd2", "eval", "bwd2", "bwd1"]


def main():
    from timevqvae.hip import _native
    from timevqvae.models.vq_vae import ResBlock
    dev = torch.device("cuda", 0)
    B = 256
    for C, W in ((8, 64), (16, 32), (32, 16)):
        m = ResBlock(C, C, False, dropout=0.3).to(dev).train()
        x = torch.randn(B, C, 3, W, device=dev, requires_grad=True)
        gy = torch.randn(B, C, 3, W, device=dev)
        tb = torch.zeros(5 * B * 16, dtype=torch.int64, device=dev)
        lib = _native.lib()
        lib.tvq_rb_timing.argtypes = [ctypes.c_void_p]
        for it in range(3):
            if it == 2:
                lib.tvq_rb_timing(ctypes.c_void_p(tb.data_ptr()))
            y = m(x)
            torch.autograd.backward(y, gy, inputs=[x] + list(m.parameters()))
            torch.cuda.synchronize()
        lib.tvq_rb_timing(ctypes.c_void_p(0))
        t = tb.view(5, B, 16).cpu().double() * 10e-3  # wall_clock64: 100 MHz -> us
        print(f"C={C} W={W}")
        for k, name in enumerate(KINDS):
            tk = t[k]
            if tk[:, 0].max() == 0:
                continue
            t0 = tk[:, 0].min()
            cols = []
            for i in range(16):
                col = tk[:, i]
                if col.max() == 0:
                    continue
                cols.append(f"m{i}: med {float((col - t0).median()):6.2f} max {float((col - t0).max()):6.2f}")
            print(f"  {name}: " + " | ".join(cols))


if __name__ == "__main__":
    main()
