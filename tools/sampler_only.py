"""bench.py's sampler leg alone (BASELINE configs[4]: 1024 trajectories, graphed batch, with
and without the FidelityEnhancer), for A/B runs and rocprofv3.
usage: python tools/sampler_only.py [reps]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "t-vq-vae-trajgen_amd"))
import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    dev = torch.device("cuda", 0)
    tr = bench.JointTrainer(dev, 1)
    print(json.dumps(bench.sampler_leg(tr, dev, reps=reps)))
