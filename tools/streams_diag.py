"""Losses of 4 joint steps: eager/graph x single/multi stream (debug aid)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "t-vq-vae-trajgen_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

import bench  # noqa: E402
from test_graph import _batch, _cfg  # noqa: E402
from timevqvae.hip import streams  # noqa: E402


def run(graph, multi, dev, batch):
    streams.ENABLED = multi
    tr = bench.JointTrainer(dev, 1, cfg=_cfg(), length=64, channels=3)
    out = []
    if graph:
        tr.capture(batch)
        out += ["w", "w"]
        n = 2
    else:
        n = 4
    for _ in range(n):
        o1, o2 = tr.step(batch)
        out.append((round(float(o1["loss"].detach().sum()), 6), round(float(o2["loss"].detach()), 4)))
    torch.cuda.synchronize()
    return out, tr.opt1.flat.clone()


def main():
    dev = torch.device("cuda", 0)
    batch = _batch(dev)
    res = {}
    for graph in (False, True):
        for multi in (False, True):
            l, p = run(graph, multi, dev, batch)
            res[(graph, multi)] = p
            print(f"graph={graph} multi={multi}: {l}", flush=True)
    base = res[(False, False)]
    for k, p in res.items():
        print(k, "params equal to eager single:", torch.equal(p, base),
              float((p - base).abs().max()))


if __name__ == "__main__":
    main()
