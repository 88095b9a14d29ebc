"""A/B of two GraphedSampler variants on one box, alternated: a module-level boolean switch
of the package flipped for variant B before its capture (each variant keeps the flag value it
was captured with: the graph holds the launches).
usage: python tools/sampler_ab.py [module:FLAG]   e.g. models.bidirectional_transformer:FUSED_SAMPLE
(no argument: the default sampler against itself, the noise floor)."""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "t-vq-vae-trajgen_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
from timevqvae.utils.sample_utils import GraphedSampler  # noqa: E402

dev = torch.device("cuda", 0)
mg = bench.JointTrainer(dev, 1).s2.maskgit.eval()
spec = sys.argv[1] if len(sys.argv) > 1 else None
variants = {"A": GraphedSampler(mg, 1024, dev)}
if spec:
    mod_name, flag = spec.split(":")
    mod = importlib.import_module("timevqvae." + mod_name)
    old = getattr(mod, flag)
    setattr(mod, flag, not old)
    variants["B"] = GraphedSampler(mg, 1024, dev)
    setattr(mod, flag, old)
else:
    variants["B"] = GraphedSampler(mg, 1024, dev)


def t(s, n=20):
    s.sample()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        s.sample()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


res = {k: [] for k in variants}
for r in range(4):
    for k, s in variants.items():
        res[k].append(t(s))
for k, v in res.items():
    print(spec, k, " ".join(f"{x:.3f}" for x in v), "min %.3f" % min(v), flush=True)
