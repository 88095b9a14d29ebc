"""Capture + replay the joint step once under the current TVQ_STREAMS_* env (debug aid)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "t-vq-vae-trajgen_amd"))
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    tr = bench.JointTrainer(dev, 1, length=64, channels=3)
    g = torch.Generator().manual_seed(5)
    batch = (torch.randn(16, 3, 64, generator=g).to(dev), torch.randint(0, 5, (16, 1)).to(dev))
    tr.capture(batch)
    o1, o2 = tr.step(batch)
    torch.cuda.synchronize()
    print(os.environ.get("TVQ_STREAMS_INLINE", "-"), "ok", float(o1["loss"].detach().sum()),
          float(o2["loss"].detach()), flush=True)


if __name__ == "__main__":
    main()
