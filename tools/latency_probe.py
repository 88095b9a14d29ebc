"""Graph-replayed time per dependent kernel for elementwise ops of the step's tensor sizes
(the floor a small conv / BN / Snake launch sits on).  usage: python tools/latency_probe.py"""
import torch


def per_kernel(fn, n=200):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 5 * 1e3 / n


def main():
    dev = torch.device("cuda", 0)
    for numel in (1024, 98304, 393216, 1572864, 4194304, 16777216):
        x = torch.zeros(numel, device=dev)
        y = torch.zeros(numel, device=dev)
        t = per_kernel(lambda: torch.add(x, 1.0, out=y))
        mb = 8 * numel / 1e6
        print(f"add {numel:9d} floats ({mb:6.2f} MB moved): {t:6.2f} us/kernel, {mb / t:6.2f} TB/s",
              flush=True)


if __name__ == "__main__":
    main()
