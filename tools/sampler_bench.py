"""Sampler throughput (BASELINE config 5): MaskGIT iterative decoding of `num` trajectories
(10 LF steps + 1 HF step) + LF/HF decoding, at the bench architecture (config B dims,
random-init weights).  usage: python tools/sampler_bench.py [num] [reps]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "t-vq-vae-trajgen_amd"))
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    num = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    dev = torch.device("cuda", 0)
    mg = bench.JointTrainer(dev, 1).s2.maskgit.eval()

    def run():
        s_l, s_h = mg.iterative_decoding(num=num, device=dev)
        x = mg.decode_token_ind_to_timeseries(s_l, "lf") + mg.decode_token_ind_to_timeseries(s_h, "hf")
        return x

    with torch.no_grad():
        run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            x = run()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps
    print(json.dumps({"metric": "MaskGIT sampling (iterative decoding + decode), trajectories/s",
                      "num": num, "ms_per_batch": round(dt * 1e3, 2),
                      "trajectories_per_s": round(num / dt, 1), "shape": list(x.shape)}))


if __name__ == "__main__":
    main()
