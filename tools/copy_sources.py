"""Attribute device copies (aten::copy_ / clone / contiguous) and every other PyTorch-native
kernel of the joint step to Python call sites with torch.profiler.
usage: python tools/copy_sources.py [sampler]"""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "t-vq-vae-trajgen_amd"))
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

import bench  # noqa: E402


def main():
    """`python tools/copy_sources.py [sampler]`: the joint step, or one sampling batch."""
    dev = torch.device("cuda", 0)
    tr = bench.JointTrainer(dev, 1)
    batch = bench.synthetic_batch(1234, dev)
    if sys.argv[1:] == ["sampler"]:
        mg = tr.s2.maskgit.eval()

        def work():
            with torch.no_grad():
                s_l, s_h = mg.iterative_decoding(num=1024, device=dev)
                mg.decode_token_ind_to_timeseries(s_l, "lf")
                mg.decode_token_ind_to_timeseries(s_h, "hf")
    else:
        def work():
            tr.step(batch)
    for _ in range(2):
        work()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        work()
        torch.cuda.synchronize()
    sites = collections.Counter()
    kern = collections.Counter()
    for ev in prof.events():
        ks = [k.name for k in getattr(ev, "kernels", [])]
        if not ks:
            continue
        for k in ks:
            kern[k[:60]] += 1
        if not any(("opy" in k or "emcpy" in k or "emset" in k or "at::native" in k) for k in ks):
            continue
        stack = [f for f in (ev.stack or []) if "site-packages" not in f and "dist-packages" not in f]
        sites[(ev.name, " | ".join(stack[:3]) if stack else "?", ks[0][:30])] += 1
    for (name, site, k), n in sites.most_common(60):
        print(f"{n:5d} {name:22s} {k:30s} {site}")
    print("--- device activity names")
    for k, n in kern.most_common(15):
        print(f"{n:5d} {k}")


if __name__ == "__main__":
    main()
