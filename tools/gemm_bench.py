"""GEMM micro-bench at the transformer's shapes (sampler batch 1024 and train batch 256):
HIP-event time per launch, achieved TFLOP/s, and the fraction of the fp32 MFMA peak.
usage: python tools/gemm_bench.py [shape names]   (TVQ_GEMM_SKINNY=0: generic kernel only)"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "t-vq-vae-trajgen_amd"))
import torch  # noqa: E402

from timevqvae.hip.linear import gemm  # noqa: E402

PEAK = 157.3

# (name, M, N, K, kind): kind nt = X W^T (fwd), nn = dY W (dX), tn = dY^T X (dW)
SHAPES = [
    ("lf_proj_sampler", 25600, 128, 128, "nt"),
    ("lf_logits_sampler", 24576, 512, 128, "nt"),
    ("hf_proj_in_sampler", 99328, 32, 256, "nt"),
    ("hf_proj_out_sampler", 99328, 256, 32, "nt"),
    ("hf_head_sampler", 98304, 128, 256, "nt"),
    ("lf_proj_train", 6400, 128, 128, "nt"),
    ("lf_dx_train", 6400, 128, 128, "nn"),
    ("lf_dw_train", 128, 128, 6400, "tn"),
    ("lf_logits_dx_train", 6144, 128, 512, "nn"),
    ("lf_logits_dw_train", 512, 128, 6144, "tn"),
    ("hf_head_dw_train", 128, 256, 24576, "tn"),
    ("hf_dx_train", 24832, 32, 64, "nn"),
    ("hf_dw_train", 32, 32, 24832, "tn"),
    ("hf_ff_dw_train", 64, 32, 24832, "tn"),
]


def main():
    dev = torch.device("cuda", 0)
    # bring the clocks up first (the chip idles at a low clock; short loops would time
    # the ramp, not the kernel)
    a = torch.randn(8192, 4096, device=dev)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.5:
        a = a @ a[:4096, :4096] * 1e-3
        torch.cuda.synchronize()
    res = []
    only = set(sys.argv[1:])  # shape names to run (all when empty)
    for name, M, N, K, kind in SHAPES:
        if only and name not in only:
            continue
        if kind == "nt":
            A = torch.randn(M, K, device=dev)
            B = torch.randn(N, K, device=dev)
            args = (A, K, 1, B, 1, K)
        elif kind == "nn":
            A = torch.randn(M, K, device=dev)
            B = torch.randn(K, N, device=dev)
            args = (A, K, 1, B, N, 1)
        else:  # C[M][N] = A^T B, A [K][M], B [K][N]
            A = torch.randn(K, M, device=dev)
            B = torch.randn(K, N, device=dev)
            args = (A, 1, M, B, N, 1)
        out = torch.empty(M, N, device=dev)
        for _ in range(3):
            gemm(*args, M, N, K, out=out, ldc=N)
        torch.cuda.synchronize()
        # time a captured graph of n launches: host launch cost (ctypes, ~10-20 us per
        # call) would otherwise set the rate of these short kernels
        n = 50
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            for _ in range(n):
                gemm(*args, M, N, K, out=out, ldc=N)
        graph.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(4):
            graph.replay()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / (4 * n) * 1e3
        tf = 2.0 * M * N * K / (us * 1e-6) / 1e12
        ref = (args[0].double().reshape(-1)[:0])  # noqa: F841 (keep the inputs alive)
        res.append({"name": name, "M": M, "N": N, "K": K, "kind": kind, "us": round(us, 2),
                    "tflops": round(tf, 2), "frac": round(tf / PEAK, 3)})
        print(json.dumps(res[-1]), flush=True)


if __name__ == "__main__":
    main()
