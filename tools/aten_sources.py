"""List every PyTorch-native device op of one eager joint step (or sampler batch) with where it
comes from: the autograd node running it (backward) or the Python call site (forward).
Views, allocations and metadata ops launch no kernel and are skipped.
usage: python tools/aten_sources.py [sampler|capture]"""
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

SILENT = ("view", "empty", "_unsafe_view", "as_strided", "t.default", "transpose", "permute",
          "unsqueeze", "squeeze", "expand", "reshape", "detach", "alias", "slice", "select",
          "split", "unbind", "set_", "resize_", "is_same_size", "lift_fresh",
          "_local_scalar_dense", "item", "new_empty", "diagonal", "unfold", "narrow", "chunk")


class Log(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.sites = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        name = str(func)
        if any(s in name for s in SILENT):
            return out
        tens = [a for a in list(args) + list((kwargs or {}).values()) if isinstance(a, torch.Tensor)]
        if not any(t.is_cuda for t in tens) and not (isinstance(out, torch.Tensor) and out.is_cuda):
            return out
        node = torch._C._current_autograd_node()
        if node is not None:
            site = "bwd:" + node.name()
        else:
            fr = [f for f in traceback.extract_stack()[:-1]
                  if "torch/" not in f.filename and "aten_sources" not in f.filename]
            site = " < ".join(f"{os.path.basename(f.filename)}:{f.lineno}" for f in fr[-3:][::-1])
        self.sites[(name, site)] += 1
        return out


def main():
    dev = torch.device("cuda", 0)
    tr = bench.JointTrainer(dev, 1)
    batch = bench.synthetic_batch(1234, dev)
    if sys.argv[1:] == ["sampler"]:
        mg = tr.s2.maskgit.eval()

        from timevqvae.hip import rng
        from timevqvae.hip.loss import add_losses

        def work():  # GraphedSampler's batch, eager
            with torch.no_grad():
                rng.advance(dev)
                s_l, s_h = mg.iterative_decoding(num=1024, device=dev)
                x_l = mg.decode_token_ind_to_timeseries(s_l, "lf")
                x_h = mg.decode_token_ind_to_timeseries(s_h, "hf")
                add_losses(x_l, x_h)
    elif sys.argv[1:] == ["capture"]:  # the ops recorded into the step graph (and warmup)
        log = Log()
        with log:
            tr.capture(batch)
        torch.cuda.synchronize()
        for (name, site), n in sorted(log.sites.items(), key=lambda x: -x[1]):
            print(f"{n:4d} {name:40s} {site}")
        return
    else:
        def work():
            tr.step(batch)
    for _ in range(2):
        work()
    torch.cuda.synchronize()
    log = Log()
    with log:
        work()
    torch.cuda.synchronize()
    for (name, site), n in sorted(log.sites.items(), key=lambda x: -x[1]):
        print(f"{n:4d} {name:40s} {site}")


if __name__ == "__main__":
    main()
