"""A/B of the joint train step (bench.JointTrainer, graph-replayed, B = 256) with a module-level
boolean of the package flipped for variant B before its capture, alternated on one box.
usage: python tools/step_ab.py module:FLAG | env:NAME=VALUE
  e.g. models.bidirectional_transformer:TIED_CE_FUSED, env:TVQ_BENCH_BANDS=LF,HF"""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "t-vq-vae-trajgen_amd"))
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda", 0)
batch = bench.synthetic_batch(1234, dev)
trs = {}
if sys.argv[1].startswith("env:"):  # env:NAME=VALUE (bench-level capture switches) for B
    name_, val_ = sys.argv[1][4:].split("=", 1)
    for name, v in (("A", None), ("B", val_)):
        if v is not None:
            os.environ[name_] = v
        tr = bench.JointTrainer(dev, 1)
        tr.capture(batch)
        trs[name] = tr
        os.environ.pop(name_, None)
    old = "unset"
else:
    mod_name, flag = sys.argv[1].split(":")
    newval = None
    if "=" in flag:  # module:NAME=INT
        flag, newval = flag.split("=")
        newval = int(newval)
    mod = importlib.import_module("timevqvae." + mod_name)
    old = getattr(mod, flag)
    for name, val in (("A", old), ("B", (not old) if newval is None else newval)):
        setattr(mod, flag, val)
        tr = bench.JointTrainer(dev, 1)
        tr.capture(batch)
        trs[name] = tr
    setattr(mod, flag, old)


def t(tr, n=40):
    for _ in range(3):
        tr.step(batch)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        tr.step(batch)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


res = {k: [] for k in trs}
for _ in range(4):
    for k, tr in trs.items():
        res[k].append(t(tr))
for k, v in res.items():
    print(sys.argv[1], k, "(A: default, B: switched)",
          " ".join(f"{x:.3f}" for x in v), "min %.3f" % min(v), flush=True)
