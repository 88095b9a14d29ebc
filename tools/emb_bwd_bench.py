"""Device time of tvq_embedding_bwd (group-by + segmented row sums) at the stage2 shapes, each
case replayed in a hipGraph (20 calls) and timed with HIP events on the graph's stream.
  cls   M = 256 class rows, V = 6, D = 256 / 128 (class embeddings, no dropout)
  tokl  M = 6144 LF tokens, V = 513, D = 128, half the rows the mask token, dropout 0.3
  tokh  M = 24576 HF tokens, V = 513, D = 128, likewise
usage: python tools/emb_bwd_bench.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "t-vq-vae-trajgen_amd"))
import torch  # noqa: E402

from timevqvae.hip import rng  # noqa: E402
from timevqvae.hip._native import call, ptr, value  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator().manual_seed(0)
CASES = [("cls256", 256, 6, 256, 0.0, -1), ("cls128", 256, 6, 128, 0.0, -1),
         ("tokl", 6144, 513, 128, 0.3, 512), ("tokh", 24576, 513, 128, 0.3, 512)]
for name, M, V, D, p, mask_id in CASES:
    idx = torch.randint(0, V - 1 if mask_id >= 0 else V, (M,), generator=g)
    if mask_id >= 0:
        idx[torch.rand(M, generator=g) < 0.5] = mask_id
    idx = idx.to(dev)
    gr = torch.randn(M, D, generator=g).to(dev)
    out = torch.zeros(V, D, device=dev)
    ws = torch.empty(value("tvq_embedding_bwd_workspace", M, V), device=dev, dtype=torch.int32)
    seed = rng.seed_tensor(dev)
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        def one():
            call("tvq_embedding_bwd", ptr(idx), M, D, ptr(gr), D, V, ptr(out), 1, mask_id, p,
                 ptr(seed), 7, ptr(ws), st.cuda_stream)
        one()
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=st):
            for _ in range(20):
                one()
        graph.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(5):
            graph.replay()
        e1.record(st)
        torch.cuda.synchronize()
    print(f"{name}: M={M} V={V} D={D} p={p}: {e0.elapsed_time(e1) * 1e3 / 100:.2f} us/call",
          flush=True)
