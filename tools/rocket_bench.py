"""ROCKET transform throughput: 1024 series x 10000 kernels at L=256
(the reference's FID/IS feature extraction, sampler.py:184-189), inputs resident on the
GPU, HIP events around the launches; the C oracle (oracle/rocket_ref.c, pthreads) on a
bounded sample of the same workload beside it.
usage: python tools/rocket_bench.py [n] [num_kernels] [reps]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "t-vq-vae-trajgen_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from timevqvae.evaluation import DeviceKernels, apply_kernels_device, generate_kernels
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    nk = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    L = 256
    dev = torch.device("cuda", 0)
    np.random.seed(0)
    k = generate_kernels(L, nk)
    X = np.cumsum(np.random.randn(n, L), axis=1)
    dk = DeviceKernels(k, dev)
    Xt = torch.from_numpy(X).to(dev)
    for _ in range(3):
        apply_kernels_device(Xt, dk)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        apply_kernels_device(Xt, dk)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    # algorithmic work: one multiply-add per in-range tap per output position
    lengths, dil, pad = k[1].astype(np.int64), k[3].astype(np.int64), k[4].astype(np.int64)
    olen = L + 2 * pad - (lengths - 1) * dil
    macs = n * float((olen * lengths).sum())  # upper bound (padding taps skipped)
    res = {"metric": "ROCKET features, series/s", "n": n, "num_kernels": nk, "L": L,
           "ms_per_batch": round(ms, 3), "series_per_s": round(n / (ms * 1e-3), 1),
           "fp64_gflop_per_batch": round(2 * macs / 1e9, 2),
           "achieved_tflops_fp64": round(2 * macs / (ms * 1e-3) / 1e12, 2),
           "peak_fp64_vector_tflops": 78.6}
    if "--no-cpu-baseline" not in sys.argv:
        from oracle import rocket_ref
        threads = int(os.environ.get("TVQ_CPU_THREADS", min(16, os.cpu_count() or 1)))
        m = min(n, 512)
        t0 = time.perf_counter()
        rocket_ref.apply_kernels(X[:m], k, threads=threads)
        dt = time.perf_counter() - t0
        res["cpu_baseline"] = {"value": round(m / dt, 1), "unit": "series/s", "cores": threads,
                               "kind": "port", "sample": f"{m} series x {nk} kernels of the same "
                               f"workload, oracle/rocket_ref.c: {dt:.2f} s"}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
