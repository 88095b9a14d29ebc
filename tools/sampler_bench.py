"""Sampler throughput (BASELINE config 5): MaskGIT iterative decoding of `num` trajectories
(10 LF steps + 1 HF step) + LF/HF decoding, at the bench architecture (config B dims,
random-init weights), with the CPU restatement's rate beside it (oracle/cpu_baseline.py
measure_sampler, a bounded sample of 256 trajectories).
usage: python tools/sampler_bench.py [num] [reps] [--no-cpu-baseline] [--graph]"""
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
    pos = [a for a in sys.argv[1:] if not a.startswith("--")]
    num = int(pos[0]) if pos else 1024
    reps = int(pos[1]) if len(pos) > 1 else 3
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
    res = {"metric": "MaskGIT sampling (iterative decoding + decode), trajectories/s",
           "num": num, "ms_per_batch": round(dt * 1e3, 2),
           "trajectories_per_s": round(num / dt, 1), "shape": list(x.shape)}
    if "--no-cpu-baseline" not in sys.argv:
        from oracle import cpu_baseline
        threads = int(os.environ.get("TVQ_CPU_THREADS", min(16, os.cpu_count() or 1)))
        s = cpu_baseline.measure_sampler(threads, num=256)
        res["cpu_baseline"] = {"value": round(256 / s, 2), "unit": "trajectories/s",
                               "cores": threads, "kind": "port",
                               "sample": f"256 trajectories (1 timed rep after 1 warmup) of "
                                         f"oracle/cpu_baseline.py measure_sampler: {s:.2f} s"}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
