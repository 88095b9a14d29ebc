"""Compare eager steps and graph replays tensor by tensor (debug aid)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "t-vq-vae-trajgen_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
from test_graph import _batch, _cfg  # noqa: E402


def snap(tr):
    d = {}
    for n, p in tr.s1.named_parameters():
        d["s1." + n] = p.detach().clone()
    for n, b in tr.s1.named_buffers():
        d["s1b." + n] = b.detach().clone()
    for n, p in tr.s2.named_parameters():
        d["s2." + n] = p.detach().clone()
    return d


def diff(a, b, tag):
    bad = [k for k in a if not torch.equal(a[k], b[k])]
    print(tag, "differ:", len(bad), bad[:12])


def main():
    dev = torch.device("cuda", 0)
    batch = _batch(dev)
    e = bench.JointTrainer(dev, 1, cfg=_cfg(), length=64, channels=3)
    snaps = [snap(e)]
    for _ in range(3):
        e.step(batch)
        snaps.append(snap(e))
    g = bench.JointTrainer(dev, 1, cfg=_cfg(), length=64, channels=3)
    diff(snaps[0], snap(g), "init")
    g.capture(batch)
    torch.cuda.synchronize()
    diff(snaps[2], snap(g), "after warmup(2)")
    g.step(batch)
    torch.cuda.synchronize()
    diff(snaps[3], snap(g), "after replay(1)")


if __name__ == "__main__":
    main()
