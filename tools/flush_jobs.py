"""The deferred weight-gradient slab sums of one captured joint step (bench.JointTrainer): per
producing stream the batch's jobs (rows P x columns N) and the bytes its band-end launch reads."""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "t-vq-vae-trajgen_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
from timevqvae.hip import _native  # noqa: E402

dev = torch.device("cuda", 0)
batch = bench.synthetic_batch(1234, dev)
tr = bench.JointTrainer(dev, 1)
with _native.plan_trace() as pt:
    tr.capture(batch)
jobs = collections.defaultdict(collections.Counter)
for line in pt.lines:
    if line.startswith("wgrad_flush st="):
        print(line)
    elif line.startswith("wgrad_flush_job"):
        st, P, N = line.split()[1:]
        jobs[st][(P, N)] += 1
for st, c in jobs.items():
    print(st)
    for (P, N), n in sorted(c.items(), key=lambda kv: -int(kv[0][0][2:]) * int(kv[0][1][2:]) * kv[1]):
        print(f"  {n:3d} x {P} {N}  {n * int(P[2:]) * int(N[2:]) * 4 / 1e6:.2f} MB")
