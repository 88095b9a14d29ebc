"""List the aten ops (i.e. non-HIP-ABI launches: adds, copies, fills, cats) one eager joint
step issues, grouped by (op, shapes) with the innermost product-code frame.
usage: python tools/aten_ops.py"""
import collections
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "t-vq-vae-trajgen_amd"))
import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

import bench  # noqa: E402

SKIP = {"aten.empty.memory_format", "aten.empty_strided.default", "aten.view.default",
        "aten.t.default", "aten.transpose.int", "aten.unsqueeze.default", "aten.squeeze.dim",
        "aten.as_strided.default", "aten.detach.default", "aten._unsafe_view.default",
        "aten.slice.Tensor", "aten.select.int", "aten.expand.default", "aten.permute.default",
        "aten.reshape.default", "aten.alias.default", "aten.empty_like.default",
        "aten.split.Tensor", "aten.unbind.int", "aten.squeeze.default", "aten.flatten.using_ints",
        "aten.is_same_size.default", "aten._local_scalar_dense.default", "aten.lift_fresh.default"}


class Count(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.c = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = str(func)
        if name not in SKIP:
            shapes = tuple(tuple(a.shape) for a in args if isinstance(a, torch.Tensor))[:3]
            site = "?"
            for fr in reversed(traceback.extract_stack()[:-1]):
                if "timevqvae" in fr.filename or "bench.py" in fr.filename:
                    site = f"{os.path.basename(fr.filename)}:{fr.lineno}:{fr.name}"
                    break
            self.c[(name, shapes, site)] += 1
        return func(*args, **(kwargs or {}))


def main():
    dev = torch.device("cuda", 0)
    tr = bench.JointTrainer(dev, 1)
    batch = bench.synthetic_batch(1234, dev)
    for _ in range(2):
        tr.step(batch)
    torch.cuda.synchronize()
    m = Count()
    with m:
        tr.step(batch)
    torch.cuda.synchronize()
    tot = sum(m.c.values())
    print(f"total aten ops (non-view) per eager step: {tot}")
    for (name, shapes, site), n in m.c.most_common():
        print(f"{n:4d}  {name:40s} {str(shapes)[:60]:60s} {site}")


if __name__ == "__main__":
    main()
