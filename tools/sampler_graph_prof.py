"""Replays of the graphed sampling batch alone (BASELINE configs[4], no FidelityEnhancer),
for rocprofv3 kernel tables / traces of exactly the timed batch.
usage: python tools/sampler_graph_prof.py [replays]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "t-vq-vae-trajgen_amd"))
import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    dev = torch.device("cuda", 0)
    mg = bench.JointTrainer(dev, 1).s2.maskgit.eval()
    from timevqvae.utils.sample_utils import GraphedSampler
    gs = GraphedSampler(mg, 1024, dev)
    gs.sample()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        gs.sample()
    torch.cuda.synchronize()
    print(f"graphed batch: {(time.perf_counter() - t0) / reps * 1e3:.3f} ms over {reps} replays")
