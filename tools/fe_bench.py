"""FidelityEnhancer eval forward at the sampler's batch (1024 x 6 x 256), configs/config.yaml
hyper-parameters, random weights: ms per batch (HIP events on the current stream)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "t-vq-vae-trajgen_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from timevqvae.models import FidelityEnhancer  # noqa: E402


def main(num=1024, reps=20):
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    fe = FidelityEnhancer(256, 6, bench.config(False)).to(dev).eval()
    x = torch.cumsum(0.1 * torch.randn(num, 6, 256, device=dev), -1)
    fe(x)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fe(x)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / reps
    print(json.dumps({"fe_ms_per_batch": round(ms, 3), "num": num,
                      "trajectories_per_s": round(num / ms * 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
