"""Attribute device copies (aten::copy_ / clone / contiguous) of the joint step to Python
call sites with torch.profiler.  usage: python tools/copy_sources.py"""
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
    dev = torch.device("cuda", 0)
    tr = bench.JointTrainer(dev, 1)
    batch = bench.synthetic_batch(1234, dev)
    for _ in range(2):
        tr.step(batch)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU], with_stack=True) as prof:
        tr.step(batch)
        torch.cuda.synchronize()
    sites = collections.Counter()
    for ev in prof.events():
        if ev.name in ("aten::copy_", "aten::clone", "aten::contiguous", "aten::to", "aten::_to_copy",
                       "aten::zero_", "aten::fill_", "aten::add_", "aten::zeros", "aten::cat",
                       "aten::index_put_", "aten::mul_"):
            stack = [f for f in (ev.stack or []) if "t-vq-vae-trajgen_amd" in f or "bench.py" in f]
            sites[(ev.name, stack[0] if stack else "?")] += 1
    for (name, site), n in sites.most_common(60):
        print(f"{n:5d} {name:18s} {site}")


if __name__ == "__main__":
    main()
