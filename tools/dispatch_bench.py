"""Graph-replay dispatch cost: N tiny kernels spread over S streams (fork at the start,
join at the end).  Prints us per kernel for each S.  usage: python tools/dispatch_bench.py"""
import torch


def run(n, s, dev):
    main = torch.cuda.current_stream()
    streams = [torch.cuda.Stream() for _ in range(s)]
    xs = [torch.zeros(1024, device=dev) for _ in range(s)]
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(main)
    with torch.cuda.stream(side):
        for _ in range(2):
            for x in xs:
                x.add_(1.0)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        cap = torch.cuda.current_stream()
        for st in streams:
            st.wait_stream(cap)
        for i in range(n):
            k = i % s
            with torch.cuda.stream(streams[k]):
                xs[k].add_(1.0)
        for st in streams:
            cap.wait_stream(st)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 10 * 1e3 / n


def main():
    dev = torch.device("cuda", 0)
    for s in (1, 2, 3, 4, 6, 8):
        print(f"streams={s}: {run(1200, s, dev):.2f} us/kernel", flush=True)


if __name__ == "__main__":
    main()
