"""Stage1 chains one at a time (config B, B=256): each band's encoder forward, full forward
and forward+backward, graph-replayed on one stream -- the chain lengths the joint step's
concurrent streams are bounded by.  usage: python tools/band_bench.py [LF|HF]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "t-vq-vae-trajgen_amd"))
import torch  # noqa: E402

import bench  # noqa: E402


def gtime(fn, reps=5):
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        for _ in range(2):
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
    from timevqvae.hip.conv import PackCache, wgrad_deferred
    from timevqvae.hip.signal import stft_encode
    from timevqvae.trainers import Stage1
    dev = torch.device("cuda", 0)
    m = Stage1(bench.T, bench.C, bench.config(False)).to(dev).train()
    x, _ = bench.synthetic_batch(1234, dev)
    packs = PackCache(dev)
    s = stft_encode(x, enc_l=True, enc_h=True, tgt_l=True, tgt_h=True)
    params = list(m.parameters())
    only = sys.argv[1] if len(sys.argv) > 1 else None  # "LF" / "HF": that band's fwd+bwd only
    for band in ("LF", "HF"):
        if only and band != only:
            continue
        enc = m.encoder_l if band == "LF" else m.encoder_h
        key = "enc_l" if band == "LF" else "enc_h"

        def f_enc():
            with packs.scope():
                enc.encode_timefreq(s[key])

        def f_fwd():
            with packs.scope():
                m._band(band, s)

        def f_fb():
            for p in params:
                p.grad = None
            with packs.scope():
                part = m._band(band, s)
                with wgrad_deferred():
                    torch.autograd.backward((part[1] + part[2]["loss"]).sum(), inputs=params)
        if only:
            print(f"{band}: fwd+bwd {gtime(f_fb):7.1f} us", flush=True)
            continue
        print(f"{band}: encoder fwd {gtime(f_enc):7.1f} us  band fwd {gtime(f_fwd):7.1f} us  "
              f"fwd+bwd {gtime(f_fb):7.1f} us", flush=True)


if __name__ == "__main__":
    main()
